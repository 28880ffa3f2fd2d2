# Prepass tile scan change: GPU parity tests, cfg4 bench line and cfg4 kernel trace.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/scan
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/scan/pytest_gpu.log 2>&1
timeout -k 10 300 python3 bench.py --config cfg4 > gpurun_out/scan/bench_cfg4.json 2> gpurun_out/scan/bench_cfg4.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/scan/prof_cfg4 -o run -- python3 $R/bench.py --config cfg4 --no-cpu-baseline --no-pipelined > $R/gpurun_out/scan/prof_cfg4.log 2>&1
