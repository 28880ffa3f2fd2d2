#!/bin/bash
# Round 5, step 36: 6-lane list-walk probe; the round-4 library against the tree in one process
# (lane/irregular probe, cfg A/B, record check); round-5 PMC passes of the lane kernels.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s36
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 200 python -u tools/lane_probe.py $A/libtkv_base.so $A/libtkv_g6.so --rounds 5 --only "257-384" > $O/g6_probe.jsonl 2>&1
echo "g6 rc=$?"
timeout -k 10 400 python -u tools/lane_probe.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 3 > $O/lane_probe_r4.jsonl 2>&1
rc=$?; echo "lane rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_multi.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_multi_r4.jsonl 2>&1
rc=$?; echo "multi rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/rec_probe.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 3 --reps 5 > $O/rec_probe_r4.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5_lanepmc.sh r5s36/lanepmc
echo done
