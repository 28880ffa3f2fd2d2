# Fresh-container check: GPU parity tests, smoke(), default bench line.
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_cfg2.json 2> gpurun_out/bench_cfg2.err
timeout -k 10 300 python3 bench.py --config cfg4 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err
