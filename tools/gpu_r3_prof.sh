#!/bin/bash
# Round-3 profiles of the current tree. The default bench command (cfg2, one stream, --no-pipelined so
# no two-stream launches enter the average) under rocprofv3 --kernel-trace --stats; then separate
# --pmc passes (one counter group per run): FETCH_SIZE and WRITE_SIZE for cfg2/cfg3/cfg4
# (roofline.traffic and the byte budget), TCC hit/miss for cfg2, FETCH_SIZE for the lane kernels
# (uniform 36 B, gapped WAL payloads).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3p
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
for cfg in cfg2 cfg3 cfg4; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    run pmc_${cfg}_${ctr} 120 rocprofv3 --pmc $ctr -d $O/pmc_${cfg}_${ctr} -o pmc --output-format csv -- $B --config $cfg --steps 5 --warmup 3 --min-warmup-ms 0 || exit 1
  done
done
run pmc_cfg2_TCC 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_cfg2_TCC -o pmc --output-format csv -- $B --steps 5 --warmup 3 --min-warmup-ms 0 || exit 1
L="python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 2"
run pmc_lane36_FETCH 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_lane36_FETCH -o pmc --output-format csv -- $L --only "uniform 36 B stride 36 base+0" || exit 1
run pmc_lane36_WRITE 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_lane36_WRITE -o pmc --output-format csv -- $L --only "uniform 36 B stride 36 base+0" || exit 1
run pmc_walpay_FETCH 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_walpay_FETCH -o pmc --output-format csv -- $L --only "irregular WAL payloads 36 B" || exit 1
run trace_lanes 200 rocprofv3 --kernel-trace --stats -d $O/trace_lanes -o run --output-format csv -- $L --only "WAL payloads 36 B" || exit 1
echo done
