#!/bin/bash
# Round-3 final profiles of the tree: kernel trace + stats of the default cfg2 bench command with one
# stream (--no-pipelined, so the stats average is the per-launch duration) and of cfg4, and one
# FETCH_SIZE pass each for cfg2 and cfg4 (one counter group per run). Output: gpurun_out/r3final/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3final
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {  # name limit command...
  local name=$1 t=$2
  shift 2
  timeout -k 10 -s KILL $t "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
B="python3 $R/bench.py --no-cpu-baseline --no-pipelined --no-more-configs --no-e2e"
run trace_cfg2 300 rocprofv3 --kernel-trace --stats -d $O/trace_cfg2 -o run --output-format csv -- $B || exit 1
run trace_cfg4 300 rocprofv3 --kernel-trace --stats -d $O/trace_cfg4 -o run --output-format csv -- $B --config cfg4 || exit 1
for cfg in cfg2 cfg4; do
  run pmc_${cfg}_FETCH_SIZE 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${cfg}_FETCH_SIZE -o pmc --output-format csv -- $B --config $cfg --steps 5 --warmup 3 --min-warmup-ms 0 || exit 1
done
echo done
