set -u
# Round-4 step 17: narrow-window record check staged through LDS (HEAD) against wal_rec_lanes
# (norecl): record parity tests on HEAD, then the record probe in one process.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s17
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_wal_records.py tests/test_gpu_lanes.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tools/ab/libtkv_norecl.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; grep "^{" $O/rec_probe.jsonl | cut -c1-200; exit $rc
