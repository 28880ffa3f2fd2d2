# Round-2 check on one MI355X: GPU parity suite, smoke, and bench lines with the driver's
# --warmup 5 --steps 20 (with and without the warm-up time floor) plus the default line.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --min-warmup-ms 0 --no-cpu-baseline > $O/bench_w5_nofloor.json 2> $O/bench.err
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_w5.json 2>> $O/bench.err
timeout -k 10 300 python3 bench.py > $O/bench_default.json 2>> $O/bench.err
