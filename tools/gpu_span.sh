# One-workgroup latency kernel for host spans (crc_span): the GPU parity suite, smoke and the per-put
# latency rows.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${SPAN_OUT:-span}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 tools/build/put_latency oracle/_ref/libref_crc32.so > $O/put_latency.jsonl 2> $O/put_latency.err
