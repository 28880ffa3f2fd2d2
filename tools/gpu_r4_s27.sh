set -u
# Round-4 step 27: in-process A/B of the group lanes' fifth granule taken from the next lane (shuf)
# against the product, over every lane_probe workload (group passes, class lists, small_gen).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s27
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_shuf.so --rounds 5 --reps 5 --lens 36 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; grep -c '"same_as_first": false' $O/lane_probe.jsonl; exit $rc
