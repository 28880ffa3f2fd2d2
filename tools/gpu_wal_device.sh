# Device WAL walk: its parity tests, the WAL/format GPU tests it now serves, then the formats bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/wal_device4
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal_device.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_wal_device.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_formats.py -x -v -m gpu -k "wal or sst" --timeout 120 --timeout-method thread > $O/pytest_wal_formats.log 2>&1
timeout -k 10 600 python3 -u tools/bench_formats.py > $O/bench_formats.jsonl 2> $O/bench_formats.err
