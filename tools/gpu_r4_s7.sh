set -u
# Round-4 step 7: whole GPU suite; then HEAD against HEAD~1 (tools/ab/libtkv_r4d.so) in one process:
# uniform lane batches (two-chain fold) and irregular batches (group thresholds, per-tile fused finish,
# stream verdict for small-dominated tiles).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s7
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4d.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 > $O/probe_all.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
