# Parity tests, then the bench lines cfg2-cfg5 and kernel traces of the cfg2/cfg4 bench commands.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
bash tools/gpu_benches.sh
