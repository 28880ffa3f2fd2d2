set -u
# Round-4 step 18: the whole GPU suite on the tree (new LDS-staged record-check tests included).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s18
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
# the record check staged through LDS against the granule kernel, once more on this box
timeout -k 10 300 python -u tools/rec_probe.py tools/ab/libtkv_norecl.so tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; exit $rc
