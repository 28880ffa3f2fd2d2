#!/bin/bash
# Per-kernel durations of the cfg4 step in two builds (kernel trace, one build per run).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for lib in libtkv_crc32.so:$R/tinykvpp_amd/libtkv_crc32.so libtkv_v1.so:$R/tools/ab/libtkv_v1.so; do
  n=${lib%%:*}; p=${lib#*:}
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv -- python3 $R/tools/ab_multi.py $p --only "cfg4 Zipf 128K" --rounds 4 > $O/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-4 $f | head -12; done
