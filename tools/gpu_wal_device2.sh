# Device WAL walk v2 (scan kernel, reused speculative counts, in-lane CRC of small records):
# parity tests, the WAL/format GPU tests, the path/timing probe under the kernel trace.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/wal_device3
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_wal_device.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_wal_device.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_formats.py -x -v -m gpu -k "wal or sst" --timeout 120 --timeout-method thread > $O/pytest_wal_formats.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/wal_probe.py > $O/wal_probe.txt 2>&1
