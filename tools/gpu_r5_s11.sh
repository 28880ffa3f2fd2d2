#!/bin/bash
# Round 5, step 11: region size and waves per SIMD; tables at LDS 0, u32 positions, buffer loads, cheaper marks: WAL tests, A/B against round 4 and the previous commit, PMC of the sweep.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s11
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal or Wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=$?; echo "pytest wal rc=$rc"; tail -2 $O/pytest_wal.log; grep -E "^FAILED|^ERROR" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so tools/ab/libtkv_r5k.so tools/ab/libtkv_r7k.so --rounds 4 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
echo done
