#!/bin/bash
# Round 5, step 20: kernel trace of a mixed irregular batch with crc_list_lanes in front.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s22
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/t128 -o run --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "irregular 128 B, 8" > $O/t128.log 2>&1
echo "t128 rc=$?"

timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/t2659 -o run --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "26-59" > $O/t2659.log 2>&1
echo "t2659 rc=$?"
echo done
