#!/bin/bash
# The seeded random sweep (tests/test_gpu_fuzz.py) re-seeded with each TKV_FUZZ_OFFSET given;
# one pytest process per offset, each under its own time limit; stops at the first failure.
# Usage: tools/gpu_fuzz_offsets.sh <name> <offset> ...; logs in gpurun_out/<name>/.
set -u
R=$GRAFT_REPO_ROOT
N=$1
shift
O=$R/gpurun_out/$N
mkdir -p $O
cd "$R"
for off in "$@"; do
  TKV_FUZZ_OFFSET=$off timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread > $O/fuzz_$off.log 2>&1
  rc=$?
  echo "offset $off rc=$rc $(tail -1 $O/fuzz_$off.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
