#!/bin/bash
# Round 5, step 3: in-process A/B of the sweep's loop shapes (tools/ab/libtkv_x*.so) against round 4.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s3
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tools/ab/libtkv_x0.so tools/ab/libtkv_x2.so tools/ab/libtkv_x3.so tools/ab/libtkv_x4.so tools/ab/libtkv_x0nf.so tools/ab/libtkv_x4nf.so --rounds 4 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep image $O/ab_wal.jsonl
echo done
