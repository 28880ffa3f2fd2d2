#!/bin/bash
# Round 5, step 35: probe of a 6-lane group walk for listed 257-384-byte blocks against the 8-lane walk.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s35
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 300 python -u tools/lane_probe.py $A/libtkv_base.so $A/libtkv_g6.so --rounds 5 --only "257-384" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
echo done
