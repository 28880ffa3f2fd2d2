# Bench lines for cfg2-cfg5 and kernel-trace profiles of the cfg2 and cfg4 bench commands (one GPU call).
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/benches
for c in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --config $c > gpurun_out/benches/bench_$c.json 2> gpurun_out/benches/bench_$c.err
done
cd /tmp && export TMPDIR=/tmp
for c in cfg2 cfg4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/benches/prof_$c -o run -- python3 $R/bench.py --config $c --no-cpu-baseline > $R/gpurun_out/benches/prof_$c.log 2>&1
done
