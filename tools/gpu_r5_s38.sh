#!/bin/bash
# Round 5, step 38: LDS-staged lane kernel with two steps' copies in flight (step j+2's copy into step
# j's buffer once its words are in registers) against one step (one process).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s38
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 400 python -u tools/lane_probe.py $A/libtkv_base.so $A/libtkv_lds2.so --rounds 5 --only "uniform" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
timeout -k 10 200 python -u tools/lane_probe.py $A/libtkv_base.so $A/libtkv_lds2.so --rounds 3 --lens 28,29,30,31,33,34,35,37,40,41,44,45,47 > $O/lane_lens.jsonl 2>&1
echo "lens rc=$?"
echo done
