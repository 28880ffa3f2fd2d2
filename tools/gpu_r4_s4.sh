set -u
# Round-4 step 4: small blocks listed by class (4/8/16-lane groups) against HEAD (tools/ab/libtkv_r4c.so);
# the whole GPU suite first.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s4
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4c.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; grep "^{" $O/probe_irregular.jsonl | cut -c1-160; exit $rc
