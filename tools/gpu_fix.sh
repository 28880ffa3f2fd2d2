set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 200 python3 tools/lat_probe.py > gpurun_out/lat.log 2>&1
timeout -k 10 300 python3 bench.py --config cfg4 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err
