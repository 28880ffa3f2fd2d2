set -u
# Round-4 step 9: listed small blocks packed back to back in lane space (seg_walk) against the class
# walks (tools/ab/libtkv_r4e.so = HEAD): small-block parity tests, then irregular batches in one process.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s9
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4e.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
