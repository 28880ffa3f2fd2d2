#!/bin/bash
# Round 5, step 32: the scatter's shape for listed batches: fused finish threshold (tiles) and a
# bounded rows_finish grid, against the product (one process).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s32
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 600 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so $A/libtkv_ff128.so $A/libtkv_ff256.so $A/libtkv_fg16.so $A/libtkv_fg32.so $A/libtkv_ff128fg32.so --rounds 4 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
echo done
