#!/bin/bash
# Round 5, step 16: first boundary prunes, far-jump boundaries wait; fix-up task per failing boundary (no reach pruning), passing over covered regions: WAL tests, A/B,
# the adversarial 1 GiB image with per-round fix-up statistics.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s15
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal or Wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=$?; echo "pytest wal rc=$rc"; tail -2 $O/pytest_wal.log; grep -E "^FAILED|^ERROR" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
timeout -k 10 240 python -u tools/wal_sweep_probe.py --reps 3 --image adv > $O/adv.log 2>&1
echo "adv rc=$?"; grep image $O/adv.log
echo done
