#!/bin/bash
# In-process A/B of library builds on one MI355X: tools/ab_multi.py (cfg2-cfg4 shapes, general and
# stream batches) and tools/lane_probe.py (WAL-record-sized blocks), each library against the first.
# Usage: tools/gpu_ab.sh <name> lib1.so lib2.so ...; output in gpurun_out/<name>/.
set -u
R=$GRAFT_REPO_ROOT
N=$1
shift
O=$R/gpurun_out/$N
mkdir -p $O
cd "$R"
timeout -k 10 400 python -u tools/ab_multi.py "$@" --rounds 8 > $O/ab_multi.jsonl 2>&1
rc=$?; echo "ab_multi rc=$rc"; grep -v amdgpu.ids $O/ab_multi.jsonl | cut -c1-200
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u tools/lane_probe.py "$@" --rounds 5 --reps 5 --only irregular > $O/lane_probe.jsonl 2>&1
rc=$?; echo "lane_probe rc=$rc"; grep -v amdgpu.ids $O/lane_probe.jsonl | cut -c1-200
exit $rc
