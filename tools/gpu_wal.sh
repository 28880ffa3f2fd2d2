#!/bin/bash
# WAL verify step on one MI355X: the WAL parity tests (device, formats, fuzz), an in-process A/B of
# the product library against the libraries given (tools/ab_wal.py: 1 GiB of small records, the 430 MB
# Zipf image), the 1 GiB values-made-of-records image per library (tools/wal_sweep_probe.py --image
# adv), and a kernel trace of the product's verifies. Usage: tools/gpu_wal.sh <name> [other.so ...];
# output in gpurun_out/<name>/.
set -u
R=$GRAFT_REPO_ROOT
N=${1:-wal}
shift
O=$R/gpurun_out/$N
mkdir -p $O
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_formats.py tests/test_gpu_fuzz.py -x -q -rA -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; fi
grep -E "fake headers|giant records|values made" $O/pytest.log | head -10
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so "$@" --rounds 8 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_wal.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
for L in tinykvpp_amd/libtkv_crc32.so "$@"; do
  timeout -k 10 200 python -u tools/wal_sweep_probe.py $L --image adv --reps 4 > $O/adv_$(basename $L .so).jsonl 2>&1
  rc=$?; echo "adv $L rc=$rc"; grep -v amdgpu.ids $O/adv_$(basename $L .so).jsonl | grep -v '"rep"' | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "${TRACE:-}" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace_wal -o run --output-format csv -- python3 $R/tools/ab_wal.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 3 > $O/trace_wal.log 2>&1
  echo "trace rc=$?"
fi
