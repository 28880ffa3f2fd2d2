#!/bin/bash
# Round 5, step 23: kernel trace of tools/dbg_list_probe.py on the product library.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s23
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace -d $O/t -o run --output-format csv -- python3 $R/tools/dbg_list_probe.py $R/tinykvpp_amd/libtkv_crc32.so > $O/t.log 2>&1
echo "t rc=$?"; cat $O/t.log | grep ms
