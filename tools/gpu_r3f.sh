#!/bin/bash
# Device WAL verify with the header-only walk and the coalesced CRC kernel: WAL parity (device tests,
# formats, WAL fuzz), then an in-process A/B against the previous build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_formats.py tests/test_gpu_fuzz.py -x -q -rA -s --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $O/ab_wal.jsonl
exit $rc
