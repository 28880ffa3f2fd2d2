# Round-2 cfg3 line (kernel, end to end from pinned host, reference CPU path) and FETCH_SIZE /
# WRITE_SIZE passes for cfg2 and cfg3 (separate runs, counters never inside the timed run).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${CFG3_OUT:-cfg3}
mkdir -p $O
timeout -k 10 400 python3 bench.py --config cfg3 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
cd /tmp && export TMPDIR=/tmp && cd $R
for c in cfg2 cfg3; do
  mkdir -p $O/pmc_$c
  for g in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $g -d $O/pmc_$c/$g -o pmc --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-pipelined --no-e2e --steps 3 --warmup 3 --min-warmup-ms 0 > $O/pmc_$c/$g.log 2>&1
  done
done
