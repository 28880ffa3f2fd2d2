set -u
# Round-4 step 16: uniform lane batches staged through LDS by LDS-DMA (HEAD) against crc_lanes_n for
# every batch (nolds): lane parity tests first (uniform every length / strides / bases / init / CRC-32C).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s16
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_nolds.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only uniform > $O/probe_uniform.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
