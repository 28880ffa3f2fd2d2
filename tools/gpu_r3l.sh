#!/bin/bash
# Region walk (wal_region): WAL parity (device tests over auto and 2 KiB regions, formats, fuzz), an
# in-process A/B against the round's first build, and a kernel trace of the verifies.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_formats.py tests/test_gpu_fuzz.py -x -q -rA -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_wal.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace_wal -o run --output-format csv -- python3 $R/tools/ab_wal.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 > $O/trace_wal.log 2>&1
echo "trace rc=$?"
