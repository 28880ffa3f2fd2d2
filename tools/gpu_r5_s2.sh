#!/bin/bash
# Round 5, step 2: WAL device tests, a kernel trace of the device verify on both images.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s2
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=$?; echo "pytest wal rc=$rc"; tail -3 $O/pytest_wal.log; grep -E "^FAILED|^ERROR" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_fuzz.log 2>&1
rc=$?; echo "pytest fuzz rc=$rc"; tail -3 $O/pytest_fuzz.log; grep -E "^FAILED|^ERROR" $O/pytest_fuzz.log | head
[ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 5 > $O/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; grep image $O/trace.log
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4 $f | head -20
echo done
