set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/b2
timeout -k 10 300 python3 bench.py > gpurun_out/b2/cfg2.json 2> gpurun_out/b2/cfg2.err
timeout -k 10 300 python3 bench.py --config cfg3 --no-e2e > gpurun_out/b2/cfg3.json 2> gpurun_out/b2/cfg3.err
timeout -k 10 300 python3 bench.py --config cfg4 > gpurun_out/b2/cfg4.json 2> gpurun_out/b2/cfg4.err
