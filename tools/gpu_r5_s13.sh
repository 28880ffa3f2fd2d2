#!/bin/bash
# Round 5, step 13: kernel trace of the device WAL verify on the 1 GiB values-made-of-records image.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s13
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 1 --image adv > $O/trace.log 2>&1
echo "trace rc=$?"; grep image $O/trace.log
echo done
