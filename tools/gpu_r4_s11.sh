set -u
# Round-4 step 11: lane kernel and narrow record check on the 64 KiB table image, two workgroups per
# CU (HEAD) against the same tree built with the 128 KiB image (l16off) and with 768-thread workgroups
# for every narrow window (l16n0); lane and record parity on HEAD first.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s11
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_wal_records.py tests/test_gpu_parity.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_l16off.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_l16n0.so --rounds 4 --reps 5 --only uniform > $O/probe_uniform.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tools/ab/libtkv_l16off.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; exit $rc
