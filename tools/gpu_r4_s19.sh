set -u
# Round-4 step 19: right-aligned lane kernel (crc_lanes_r): lane/parity/fuzz tests, then an in-process
# A/B against the build before it (lr0) and with it ahead of the LDS-staged kernel (lr2).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s19
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_lr2.so --rounds 5 --reps 5 --only uniform > $O/lane_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
