#!/bin/bash
# Round 5, step 5: 10 KiB regions on the 64 KiB table image: WAL tests, A/B of region sizes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s5
mkdir -p $O
cd $R
#timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal or Wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=0; echo "pytest wal rc=$rc"; tail -2 $O/pytest_wal.log; grep -E "^FAILED|^ERROR" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_r10a3.so --rounds 4 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
echo done
