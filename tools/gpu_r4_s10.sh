set -u
# Round-4 step 10: the lane kernel on a 64 KiB 16-replica table image with two workgroups per CU
# (l16a: 1024 threads DEPTH 2; l16b: 768 threads DEPTH 3; l16c: 1024 threads DEPTH 3, conflicts only)
# against the product, uniform batches in one process; lane parity with l16a/l16b loaded as the library.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s10
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_l16a.so tools/ab/libtkv_l16b.so tools/ab/libtkv_l16c.so --rounds 4 --reps 5 --only uniform > $O/probe_uniform.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
