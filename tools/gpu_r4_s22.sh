set -u
# Round-4 step 22: right-aligned lanes with the load pipeline intact (keep_live): lane/parity/fuzz tests,
# then in-process A/B: lr0 (before right-aligned lanes), product (lengths that are not whole dwords),
# rall (every length, ahead of the LDS-staged kernel).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s22
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_small_gen.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_rall.so --rounds 5 --reps 5 --only uniform --lens 5,10,16,17,18,19,20,21,22,23,24,25,26,27,28,32,33,36,40,48,49,50,51,53,55,57,59,61,63 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
