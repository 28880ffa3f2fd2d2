#!/bin/bash
# Single-pass irregular prepass + the WAL verify redesign: the whole GPU suite, then in-process A/Bs
# (WAL verify and the irregular shapes, the prepass on and off) against the round's first build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep -v amdgpu.ids $O/ab_wal.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_multi_1p.jsonl 2>&1
rc=$?; echo "ab_multi 1p rc=$rc"; grep -v amdgpu.ids $O/ab_multi_1p.jsonl
if [ $rc -ne 0 ]; then exit $rc; fi
TKV_PREPASS_1P=0 timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_multi_3k.jsonl 2>&1
rc=$?; echo "ab_multi 3k rc=$rc"; grep -v amdgpu.ids $O/ab_multi_3k.jsonl
exit $rc
