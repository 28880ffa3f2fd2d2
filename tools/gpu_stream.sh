# Stream mode (byte-stream row walk for back-to-back irregular batches): its tests, the irregular
# parity tests, an in-process comparison with the builds in tools/ab/, and the cfg4 bench under the
# kernel trace.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${STREAM_OUT:-stream}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_stream.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "irregular or zipf or small or shards or tiles or prepass" --timeout 300 --timeout-method thread > $O/pytest_irr.log 2>&1
timeout -k 10 600 python3 tools/ab_multi.py --no-check tinykvpp_amd/libtkv_crc32.so tools/ab/*.so > $O/ab.jsonl 2> $O/ab.err
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config cfg4 --steps 20 --warmup 20 --no-cpu-baseline > $O/bench_cfg4.json 2> $O/bench_cfg4.err
bash tools/pmc_cmd.sh $R/$O/pmc tools/stream_vs_packed.py --reps 10
