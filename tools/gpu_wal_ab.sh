# Device WAL verify: the WAL GPU tests on the product build, then an in-process A/B against the
# builds in tools/ab/ (tools/ab_wal.py).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${WAL_OUT:-walab}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_formats.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_wal.log 2>&1
timeout -k 10 600 python3 -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/*.so > $O/ab.jsonl 2> $O/ab.err
