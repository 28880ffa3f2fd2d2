set -u
# Round-4 step 33: the whole GPU suite on the product (walks with one step in flight), then the
# combined change against the build before it (prewl) on the irregular workloads.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s33
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/lane_probe.py tools/ab/libtkv_prewl.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 --only irregular > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
