#!/bin/bash
# Lane-kernel pipeline shapes (in-process A/B) and the per-tile lane density change.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lanes.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest_lanes.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so tools/ab/libtkv_d3i1.so tools/ab/libtkv_d4u1.so tools/ab/libtkv_d2i1.so tools/ab/libtkv_r2.so --rounds 3 --reps 3 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 50 --warmup 20 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 $O/bench.json
exit $rc
