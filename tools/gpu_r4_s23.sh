set -u
# Round-4 step 23: small_gen per-block registers prefetched (small_gen/lanes tests), then in-process A/B:
# right-aligned lanes at 49-63 B by pipeline depth (product 4, rd1/rd2/rd3), and per-block-register
# uniform batches of 65 B - 2 KiB against the build before the prefetch (lr0).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s23
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_small_gen.py tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_rd1.so tools/ab/libtkv_rd2.so tools/ab/libtkv_rd3.so --rounds 5 --reps 5 --only "uniform 5" --lens 49,50,51,53,55,57,59,61,63 > $O/depth_probe.jsonl 2>&1
rc=$?; echo "depth rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 --only uniform --init --lens 26,59,100,200,300,500,1000,2000 > $O/init_probe.jsonl 2>&1
rc=$?; echo "init rc=$rc"; exit $rc
