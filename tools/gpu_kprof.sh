#!/bin/bash
# Per-kernel durations of one ab_multi workload for each library (one process per library, so the
# kernel names do not mix): rocprofv3 --kernel-trace --stats. Usage: tools/gpu_kprof.sh <name>
# <workload substring> lib1.so lib2.so ...; output in gpurun_out/<name>/<lib>/.
set -u
R=$GRAFT_REPO_ROOT
N=$1
W=$2
shift 2
O=$R/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in "$@"; do
  b=$(basename $L .so)
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/$b -o run --output-format csv -- python3 $R/tools/${SCRIPT:-ab_multi.py} $R/$L --only "$W" --rounds 3 ${EXTRA---no-check} > $O/$b.log 2>&1
  rc=$?; echo "$b rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/$b.log; exit $rc; fi
  f=$(find $O/$b -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-5 "$f" | cut -c1-160
done
