set -u
# Round-4 step 3: the exact-window deeper lane kernel and the deeper record pipeline against the
# previous build (tools/ab/libtkv_r4pre.so = HEAD before them), parity tests of both.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s3
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_wal_records.py tests/test_gpu_parity.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4pre.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only uniform > $O/probe_uniform.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tools/ab/libtkv_r4pre.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; grep -v amdgpu $O/rec_probe.jsonl | cut -c1-200; exit $rc
