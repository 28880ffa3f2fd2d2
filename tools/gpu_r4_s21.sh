set -u
# Round-4 step 21: right-aligned lanes for lengths that are not whole dwords: lane/parity/fuzz tests,
# then an in-process A/B against the build before them (lr0) over lengths of every tail class.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s21
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_small_gen.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 --only uniform --lens 5,10,17,18,19,21,22,23,25,26,27,49,50,51,53,55,57,59,61,63 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
