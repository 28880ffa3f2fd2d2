#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of the device WAL verify: the 1 GiB small-record and
# 430 MB Zipf images (tools/ab_wal.py) and the 1 GiB values-made-of-records image
# (tools/wal_sweep_probe.py --image adv), product library only. Usage: tools/gpu_wal_trace.sh <name>
set -u
R=$GRAFT_REPO_ROOT
N=${1:-wal_trace}
O=$R/gpurun_out/$N
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/trace_ab -o run --output-format csv -- python3 $R/tools/ab_wal.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 3 > $O/trace_ab.log 2>&1
rc=$?; echo "trace ab rc=$rc"; f=$(find $O/trace_ab -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | cut -c1-150
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $O/trace_adv -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py $R/tinykvpp_amd/libtkv_crc32.so --image adv --reps 2 > $O/trace_adv.log 2>&1
rc=$?; echo "trace adv rc=$rc"; f=$(find $O/trace_adv -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | cut -c1-150
exit $rc
