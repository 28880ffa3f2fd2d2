#!/bin/bash
# Round 5, step 4: PMC passes and a kernel trace of the sweep (x4 = product shape, x4nf = no folds).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s4
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/ab_wal.py tools/ab/libtkv_x4.so tools/ab/libtkv_x0.so --rounds 3 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
cd /tmp && export TMPDIR=/tmp
for v in x4 x4nf; do
  timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py $R/tools/ab/libtkv_$v.so --reps 3 --image small > $O/trace_$v.log 2>&1
  echo "trace $v rc=$?"
  i=0
  for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "FETCH_SIZE"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $g -d $O/pmc_${v}_$i -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py $R/tools/ab/libtkv_$v.so --reps 2 --image small > $O/pmc_${v}_$i.log 2>&1
    echo "pmc $v $i rc=$?"
  done
done
echo done
