#!/bin/bash
# Check of the current tree on one MI355X: the whole -m gpu suite, smoke(), and the default bench
# line (cfg2 value + more_configs). Usage: tools/gpu_check.sh <name>; output in gpurun_out/<name>/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-check}
mkdir -p $O
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rA --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cat $O/bench.json
exit $rc
