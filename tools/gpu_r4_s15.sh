set -u
# Round-4 step 15: lane pipeline depth for 3-granule windows (product 6; d3_7, d3_4), uniform batches.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s15
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_d3_7.so tools/ab/libtkv_d3_4.so --rounds 5 --reps 5 --only uniform > $O/probe_uniform.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
