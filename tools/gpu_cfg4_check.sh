set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_cfg4_a.json 2> gpurun_out/bench_cfg4_a.err
timeout -k 10 300 python3 tools/explore.py --irregular --rounds 3 > gpurun_out/irr_ab.log 2>&1
timeout -k 10 300 python3 bench.py --config cfg4 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_cfg4_b.json 2> gpurun_out/bench_cfg4_b.err
