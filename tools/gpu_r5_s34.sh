#!/bin/bash
# Round 5, step 34: scatter change under test (lanes, stream, irregular, fuzz), then the tile scan's
# grid (tiles looped by at most 2/4/8 workgroups per CU) against the product and the build before.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s34
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
A=tools/ab
timeout -k 10 600 python -u tools/lane_probe.py $A/libtkv_prev.so $A/libtkv_s0.so $A/libtkv_s2.so $A/libtkv_s4.so $A/libtkv_s8.so --rounds 4 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
timeout -k 10 300 python -u tools/ab_multi.py $A/libtkv_prev.so $A/libtkv_s0.so $A/libtkv_s4.so --rounds 6 > $O/ab_multi.jsonl 2>&1
echo "multi rc=$?"
echo done
