# Bench lines with one event pair around the timed region (no per-step markers), cfg2-cfg5, and the
# native kernel trace of the cfg2 and cfg4 bench commands.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ne
for c in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/ne/bench_$c.json 2> gpurun_out/ne/bench_$c.err
done
cd /tmp && export TMPDIR=/tmp
for c in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ne/prof_$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline --no-pipelined > $R/gpurun_out/ne/prof_$c.log 2>&1
done
