# Round-2 re-check of the current tree on one MI355X: full GPU parity suite, smoke, the default
# bench line under the kernel trace, cfg4 (stream mode) and cfg5 lines, and FETCH_SIZE / WRITE_SIZE
# passes for cfg4 and cfg5 (roofline.traffic).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${R2S3_OUT:-r2s3}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg2 -o run --output-format csv -- python3 bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python3 bench.py --config cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 400 python3 bench.py --config cfg5 --steps 50 --warmup 20 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
for c in cfg4 cfg5; do
  mkdir -p $O/pmc_$c
  for g in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $g -d $O/pmc_$c/$g -o pmc --output-format csv -- python3 bench.py --config $c --no-cpu-baseline --no-pipelined --steps 3 --warmup 3 --min-warmup-ms 0 > $O/pmc_$c/$g.log 2>&1
  done
done
