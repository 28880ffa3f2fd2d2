#!/bin/bash
# Round-3 GPU step: lane-kernel parity, small-block probe against the round-2 build, full GPU suite.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -x -q --timeout 120 --timeout-method thread > $O/pytest_lanes.log 2>&1
rc=$?; echo "lanes rc=$rc"; tail -3 $O/pytest_lanes.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_r2.so --rounds 3 --reps 3 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"
if [ $rc -ne 0 ]; then tail -5 $O/lane_probe.jsonl; exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "all rc=$rc"; tail -3 $O/pytest_gpu.log
exit $rc
