#!/bin/bash
# Round-5 PMC passes on the lane / group kernels: for each workload of
# tools/lane_probe.py, one rocprofv3 --pmc run per counter group (no trace domains mixed in).
# Usage: tools/gpu_r5_lanepmc.sh OUTNAME [lib.so]; output in gpurun_out/OUTNAME/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
LIB=${2:-tinykvpp_amd/libtkv_crc32.so}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$R"
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
G2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT GRBM_COUNT"
G3="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
G4="FETCH_SIZE"
i=0
for W in "uniform 26 B stride 26 base+0" "uniform 36 B stride 36 base+0" "uniform 36 B stride 44 base+8" "irregular WAL payloads 36 B"; do
  i=$((i+1))
  g=0
  for G in "$G1" "$G2" "$G3" "$G4"; do
    g=$((g+1))
    timeout -k 10 120 rocprofv3 --pmc $G -d $O/w${i}_g$g -o pmc --output-format csv -- \
      python3 tools/lane_probe.py $LIB --only "$W" --rounds 1 --reps 3 > $O/w${i}_g$g.log 2>&1
    rc=$?
    echo "w$i ($W) g$g rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $O/w${i}_g$g.log; exit $rc; fi
  done
done
