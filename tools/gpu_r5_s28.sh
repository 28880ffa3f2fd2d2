#!/bin/bash
# Round 5, step 28: crc_list_lanes: flag polls every 4 vs 64 step groups (A/B), SQ counters.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s28
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_lp64.so --rounds 5 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $g -d $O/pmc_$i -o pmc --output-format csv -- python3 $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 2 --only "irregular WAL payloads 36" > $O/pmc_$i.log 2>&1
  echo "pmc $i rc=$?"
done
echo done
