#!/bin/bash
# Round 5, step 30: crc_lanes_win (uniform lane blocks, register-staged windows): tests, A/B vs HEAD.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s30
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 --only "uniform" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
echo done
