#!/bin/bash
# Round-5 evidence on the tree, part 2: the round-4 library (tools/build_at.sh 9458629 r4) against the
# tree in one process (device WAL verify, lane/irregular probe, cfg A/B, record check), the adversarial
# WAL image, and the round-5 lane-kernel PMC passes. Output: gpurun_out/r5final2/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5final2
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 300 python -u tools/ab_wal.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 4 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep image $O/ab_wal.jsonl | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/wal_sweep_probe.py --reps 3 --image adv > $O/wal_adv.jsonl 2>&1
rc=$?; echo "wal_adv rc=$rc"; tail -2 $O/wal_adv.jsonl | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 3 > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane_probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ab_multi.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_multi.jsonl 2>&1
rc=$?; echo "ab_multi rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/rec_probe.py $A/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 3 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec_probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5_lanepmc.sh r5final2/lanepmc
echo done
