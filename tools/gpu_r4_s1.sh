set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s1
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_gpu_wal_records.py tests/test_gpu_wal_device.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
# rc 1 = some tests failed (nothing crashed): the measurements below still run and check their own results
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_multi.py tools/ab/libtkv_r4base.so tinykvpp_amd/libtkv_crc32.so --rounds 10 --only cfg4 > $O/ab_finish.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu $O/ab_finish.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tools/ab/libtkv_r4base.so tinykvpp_amd/libtkv_crc32.so --rounds 3 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 3 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; grep -v amdgpu $O/rec_probe.jsonl | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so:walk=0 tinykvpp_amd/libtkv_crc32.so:walk=1 --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep -v amdgpu $O/ab_wal.jsonl | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/walk_probe.py --rounds 3 > $O/walk_probe.jsonl 2>&1
rc=$?; echo "walk rc=$rc"; grep -v amdgpu $O/walk_probe.jsonl | cut -c1-250
exit $rc
