#!/bin/bash
# Round-5 evidence on the tree, part 1: the GPU suite, smoke(), the default bench line, kernel traces of
# cfg2 (one stream: the stats average is the per-launch duration), cfg4 and the device WAL verify, one
# FETCH_SIZE pass each for cfg2-cfg5 and the WAL verify, SQ passes of the WAL sweep. Part 2 (the probes
# against the round-4 library, lane PMC): tools/gpu_r5_final2.sh. Output: gpurun_out/r5final/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5final
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $O/bench.json; [ $rc -eq 0 ] || exit $rc
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
run trace_wal 300 rocprofv3 --kernel-trace --stats -d $O/trace_wal -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 5 || exit 1
for cfg in cfg2 cfg3 cfg4 cfg5; do
  run pmc_${cfg}_FETCH_SIZE 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${cfg}_FETCH_SIZE -o pmc --output-format csv -- $B --config $cfg --steps 5 --warmup 3 --min-warmup-ms 0 || exit 1
done
run pmc_wal_FETCH_SIZE 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_wal_FETCH_SIZE -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 2 --image small || exit 1
run pmc_wal_sq1 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $O/pmc_wal_sq1 -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 2 --image small || exit 1
run pmc_wal_sq2 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH -d $O/pmc_wal_sq2 -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 2 --image small || exit 1
echo done
