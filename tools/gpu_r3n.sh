#!/bin/bash
# wal_region counters (separate --pmc passes over one verify of each image) and an A/B against a
# probe build without the LDS fold (tools/ab/libtkv_nofold.so).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3n
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_nofold.so tools/ab/libtkv_v1.so --rounds 6 > $O/ab_wal.jsonl 2>&1 || exit 1
grep -v amdgpu.ids $O/ab_wal.jsonl
cd /tmp && export TMPDIR=/tmp
P="python3 $R/tools/ab_wal.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 1"
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/p1 -o pmc --output-format csv -- $P > $O/p1.log 2>&1 || exit 1
echo p1 ok
timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $O/p2 -o pmc --output-format csv -- $P > $O/p2.log 2>&1 || exit 1
echo p2 ok
timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p3 -o pmc --output-format csv -- $P > $O/p3.log 2>&1 || exit 1
echo p3 ok
timeout -k 10 -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d $O/p4 -o pmc --output-format csv -- $P > $O/p4.log 2>&1 || exit 1
echo p4 ok
