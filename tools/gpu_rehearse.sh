set -e
cd $GRAFT_REPO_ROOT
export TKV_BENCH_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 50 --warmup 20 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --steps 20 --warmup 10 --config cfg4 > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err
