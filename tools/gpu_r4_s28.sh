set -u
# Round-4 step 28: the whole GPU suite on the product (16-lane list walk with the neighbour granule),
# then in-process A/B against the same build without it (g16off) on the irregular workloads.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s28
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/lane_probe.py tools/ab/libtkv_g16off.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 --only irregular > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
