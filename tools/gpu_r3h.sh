#!/bin/bash
# Single-pass prepass with the unrolled scatter (A/B on and off against the round's first build), a
# kernel trace of the device WAL verify, and the FETCH_SIZE calibration of the packed load pattern.
set -u
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3h
mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_lanes.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_multi_1p.jsonl 2>&1 || exit 1
grep -v amdgpu.ids $O/ab_multi_1p.jsonl
TKV_PREPASS_1P=0 timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_multi_3k.jsonl 2>&1 || exit 1
grep -v amdgpu.ids $O/ab_multi_3k.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace_wal -o run --output-format csv -- python3 $R/tools/ab_wal.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 > $O/trace_wal.log 2>&1 || exit 1
echo "trace_wal ok"
bash $R/tools/gpu_r3_calib.sh
