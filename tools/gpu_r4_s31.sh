set -u
# Round-4 step 31: packed kernel with its first loads ahead of the table fill: parity tests, then
# in-process A/B against the fill-first build (pkold) on cfg2 and the 64 KiB packed batch, twice.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s31
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_multi.py tools/ab/libtkv_pkold.so tinykvpp_amd/libtkv_crc32.so --rounds 10 --only packed > $O/ab_multi.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_pkold.so --rounds 10 --only packed > $O/ab_multi2.jsonl 2>&1
rc=$?; echo "ab2 rc=$rc"; exit $rc
