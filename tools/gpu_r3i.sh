#!/bin/bash
# Packed kernel's pipeline tail: loads past a wave's range read the dummy buffer instead of reloading
# the last row (probe build tools/ab/libtkv_noreload.so). Rate A/B in one process, then a FETCH_SIZE
# pass of the cfg2 shape for each library.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3i
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_multi.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_noreload.so --rounds 8 > $O/ab_multi.jsonl 2>&1 || exit 1
grep -v amdgpu.ids $O/ab_multi.jsonl
cd /tmp && export TMPDIR=/tmp
for L in libtkv_crc32:$R/tinykvpp_amd/libtkv_crc32.so noreload:$R/tools/ab/libtkv_noreload.so; do
  n=${L%%:*}; f=${L#*:}
  timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$n -o pmc --output-format csv -- python3 $R/tools/ab_multi.py $f --rounds 1 --reps 3 --only "cfg2" > $O/fetch_$n.log 2>&1 || exit 1
  echo "fetch $n ok"
done
