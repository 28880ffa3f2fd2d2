#!/bin/bash
# Stream-mode finish folded into crc_stream: stream/irregular parity, then an in-process A/B of cfg2,
# cfg4 and the other irregular shapes against the previous build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_lanes.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 8 > $O/ab_multi.jsonl 2>&1
rc=$?; echo "ab rc=$rc"; cat $O/ab_multi.jsonl | grep -v amdgpu.ids
exit $rc
