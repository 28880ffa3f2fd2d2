set -u
# Round-4 step 14: the tile scan's last workgroup scans the tile sums (HEAD) against every scatter
# workgroup summing them (noticket): prepass-path parity tests on HEAD, then irregular batches and
# cfg4 / 64 KiB stream batches in one process.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s14
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_noticket.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py tools/ab/libtkv_noticket.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_libs.jsonl 2>&1
rc=$?; echo "ab_libs rc=$rc"; grep "^{" $O/ab_libs.jsonl | cut -c1-300; exit $rc
