set -u
# Round-4 step 30: lane tests on the product (LDS-staged lanes leave the previous store in flight), then
# in-process A/B against the build that waits for it (lswait) on 28-47-byte uniform blocks.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s30
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tools/ab/libtkv_lswait.so tinykvpp_amd/libtkv_crc32.so --rounds 7 --reps 5 --only "uniform" --lens 28,30,33,36,40,44,47 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
