#!/bin/bash
# Round 5, step 18: kernel traces of irregular WAL-payload batches (36 B with 8-byte gaps; 180-400 B)
# to split their time between the prepass and the phases.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s18
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/t36 -o run --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "irregular WAL payloads 36" > $O/t36.log 2>&1
echo "t36 rc=$?"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/t180 -o run --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "180-400" > $O/t180.log 2>&1
echo "t180 rc=$?"
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/tu36 -o run --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "36 B stride 44" > $O/tu36.log 2>&1
echo "tu36 rc=$?"
echo done
