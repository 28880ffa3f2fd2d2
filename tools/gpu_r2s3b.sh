# cfg4 step under the kernel trace (per-kernel breakdown of the timed steps), and the bench's
# multi-rank code path over RCCL at WORLD_SIZE 1 (TKV_BENCH_FORCE_DIST=1 under torch.distributed.run).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${R2S3_OUT:-r2s3b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run --output-format csv -- python3 bench.py --config cfg4 --no-cpu-baseline --no-pipelined > $O/bench_cfg4.json 2> $O/bench_cfg4.err
TKV_BENCH_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nccl_ws1.json 2> $O/bench_nccl_ws1.err
