set -u
# Round-4 step 29: record-check tests on the product (LDS-staged record check no longer waits for the
# previous step's store), then in-process A/B against the build that waits (recsw).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s29
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_records.py tests/test_gpu_wal_device.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tools/ab/libtkv_recsw.so tinykvpp_amd/libtkv_crc32.so --rounds 7 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; exit $rc
