set -u
# Round-4 step 25: the whole GPU suite on the product (right-aligned lanes, 5-granule windows without
# prefetch), the record check's 4-granule kernel by steps in flight (3 product, 0, 1), and the uniform
# lane lengths against the build before right-aligned lanes (lr0).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s25
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_rec4a0.so tools/ab/libtkv_rec4a1.so --rounds 5 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_lr0.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 --only uniform --lens 5,10,16,17,21,26,27,28,33,36,48,49,52,53,56,59,60,63 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
