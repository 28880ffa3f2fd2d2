set -u
# Round-4 step 32: steps in flight for the irregular walks: lane/group passes with one step (walk1,
# product 2), class-list walks with one or two (list1, list2; product 3); in-process A/B on the
# irregular lane_probe workloads.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s32
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_walk1.so tools/ab/libtkv_list1.so tools/ab/libtkv_list2.so --rounds 5 --reps 5 --only irregular > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; exit $rc
