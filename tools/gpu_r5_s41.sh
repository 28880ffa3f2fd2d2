#!/bin/bash
# Round 5, step 41: kernel split of the gated lane-only batch (gapped 36-byte WAL payloads) and of a
# batch that falls through the one-pass kernel (gapped 100-200 B) on the final tree.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s41
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for w in "payloads 36 B" "payloads 100-200 B"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t$i -o run --output-format csv -- python3 -u $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 5 --only "$w" > $O/t$i.log 2>&1
  rc=$?; echo "$w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo done
