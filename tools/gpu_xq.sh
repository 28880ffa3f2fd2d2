set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --config cfg4 > gpurun_out/bench_cfg4.json 2> gpurun_out/bench_cfg4.err
timeout -k 10 300 python3 bench.py --config cfg5 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err
timeout -k 10 400 python3 tools/bench_formats.py > gpurun_out/bench_formats.jsonl 2> gpurun_out/bench_formats.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg4 -o run -- python3 $R/bench.py --config cfg4 --no-cpu-baseline > $R/gpurun_out/prof_cfg4.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg2 -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_cfg2.log 2>&1
