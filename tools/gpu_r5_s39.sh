#!/bin/bash
# Round 5, step 39: cfg4's small launches: the stream finish with the predecessor's end and wave loaded
# directly (fd), the tile scan's offsets loaded with the lengths in the 1024-thread shape (oe), both
# (fdoe): in-process cfg A/B, listed batches, and a kernel trace of cfg4 per build.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s39
mkdir -p $O
cd $R
A=tools/ab
timeout -k 10 300 python -u tools/ab_multi.py $A/libtkv_base.so $A/libtkv_fd.so $A/libtkv_oe.so $A/libtkv_fdoe.so --rounds 8 > $O/ab_multi.jsonl 2>&1
echo "multi rc=$?"
timeout -k 10 300 python -u tools/lane_probe.py $A/libtkv_base.so $A/libtkv_oe.so --rounds 4 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
cd /tmp && export TMPDIR=/tmp
for v in base fd oe fdoe; do
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/t_$v -o run --output-format csv -- python3 $R/tools/ab_multi.py $R/tools/ab/libtkv_$v.so --rounds 3 --only "cfg4 Zipf 128K" > $O/t_$v.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
