# Merged irregular row kernel (crc_irregular): stream and irregular parity tests on the product
# build, in-process A/B against the two-kernel build and pipeline-shape variants (tools/ab/), and the
# per-put latency rows with the host span path.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${MERGE_OUT:-merge}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_stream.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_stream.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_formats.py tests/test_gpu_wal_device.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_irr.log 2>&1
timeout -k 10 600 python3 tools/ab_multi.py --rounds 10 tinykvpp_amd/libtkv_crc32.so tools/ab/*.so > $O/ab.jsonl 2> $O/ab.err
timeout -k 10 120 tools/build/put_latency oracle/_ref/libref_crc32.so > $O/put_latency.jsonl 2> $O/put_latency.err
