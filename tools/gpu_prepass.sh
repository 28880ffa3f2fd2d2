# Stream-mode prepass/finish changes: stream + irregular parity tests, in-process A/B against the
# previous build (tools/ab/), the cfg4 step under the kernel trace, and the bench's RCCL path at
# WORLD_SIZE 1 with the communicator built before warm-up.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${PP_OUT:-prepass}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_stream.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_formats.py tests/test_gpu_wal_device.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_irr.log 2>&1
timeout -k 10 600 python3 tools/ab_multi.py --rounds 10 --only cfg4 tinykvpp_amd/libtkv_crc32.so tools/ab/*.so > $O/ab.jsonl 2> $O/ab.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg4 -o run --output-format csv -- python3 bench.py --config cfg4 --no-cpu-baseline --no-pipelined > $O/bench_cfg4.json 2> $O/bench_cfg4.err
TKV_BENCH_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_nccl_ws1.json 2> $O/bench_nccl_ws1.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_cfg2_w5.json 2> $O/bench_cfg2_w5.err
