#!/bin/bash
# Round 5, step 33: scatter shape sweep (fused-finish tile threshold x rows_finish grid per CU).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s33
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 600 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so $A/libtkv_a.so $A/libtkv_b.so $A/libtkv_c.so $A/libtkv_d.so $A/libtkv_e.so --rounds 4 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so $A/libtkv_a.so --rounds 6 > $O/ab_multi.jsonl 2>&1
echo "multi rc=$?"
echo done
