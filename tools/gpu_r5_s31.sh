#!/bin/bash
# Round 5, step 31: kernel split of the listed mixed-class batches and of the gapped WAL payloads.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s31
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for w in "180-400" "300-1000" "100-700" "payloads 36 B"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t$i -o run -- python3 -u $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 5 --only "$w" > $O/t$i.log 2>&1
  rc=$?; echo "$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
