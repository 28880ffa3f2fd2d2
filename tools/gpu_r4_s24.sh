set -u
# Round-4 step 24: product (5-granule right-aligned windows without prefetch) tests, then in-process A/B
# of the product against nopf (no step in flight in crc_lanes_n 4-5 granule windows, crc_packed_small_gen,
# the lane/group/list walks and the record check's granule kernel) over every lane_probe workload and
# the record probe.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s24
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_small_gen.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_nopf.so --rounds 5 --reps 5 --lens 16,26,36,48,52,56,59,60 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_nopf.so --rounds 5 --reps 5 --only uniform --init --lens 26,52,59 > $O/init_probe.jsonl 2>&1
rc=$?; echo "init rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_nopf.so --rounds 5 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; exit $rc
