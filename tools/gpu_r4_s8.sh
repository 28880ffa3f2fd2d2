set -u
# Round-4 step 8: HEAD (group thresholds 3072 / 3968, stream verdict for small-dominated tiles) against
# tools/ab/libtkv_r4d.so (before them) in one process: irregular lane_probe batches and the stream /
# cfg batches of tools/ab_libs.py; then the GPU tests that pin the verdict.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s8
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4d.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_libs.py tools/ab/libtkv_r4d.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_libs.jsonl 2>&1
rc=$?; echo "ab_libs rc=$rc"; grep -v amdgpu $O/ab_libs.jsonl | cut -c1-300; exit $rc
