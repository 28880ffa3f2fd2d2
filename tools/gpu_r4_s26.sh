set -u
# Round-4 step 26: record/lane tests on the product (4-granule record windows at the fold), then
# in-process A/B for 26-47-byte uniform blocks: product, LDS-staged kernel without prefetch (ldsnp),
# right-aligned windows for every length with 3-4 granule windows at the fold (r3d1) or pipelined (r3d6).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s26
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_records.py tests/test_gpu_lanes.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_ldsnp.so tools/ab/libtkv_r3d1.so tools/ab/libtkv_r3d6.so --rounds 5 --reps 5 --only "B stride" --lens 21,26,28,30,32,33,35,36,40,44,47 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
