#!/bin/bash
# Round 5, step 1: the single-read WAL verify (wal_sweep) on the GPU: its tests, the WAL fuzz sweep,
# then the in-process A/B against the round-4 library on the 1 GiB small-record and Zipf images.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s1
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py -m gpu -v -s --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=$?; echo "pytest wal rc=$rc"; tail -3 $O/pytest_wal.log; grep -E "^FAILED|^ERROR|passed|failed" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_fuzz.log 2>&1
rc=$?; echo "pytest fuzz rc=$rc"; tail -3 $O/pytest_fuzz.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; cat $O/ab_wal.jsonl
echo done
