# Round-end rehearsal on one GPU: parity tests, smoke, the default bench command, a 2-rank gloo run.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/validate
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/validate/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/validate/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/validate/bench.json 2> gpurun_out/validate/bench.err
export TKV_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 20 > gpurun_out/validate/rehearse2.json 2> gpurun_out/validate/rehearse2.err
