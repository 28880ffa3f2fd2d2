# Device WAL verify on 1 GiB of small records: kernel trace, then PMC passes (one counter group per
# rocprofv3 run, no trace domains) to see what bounds the speculative walk.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${WAL_OUT:-walpmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 -u tools/wal_dev_probe.py 5 > $O/trace.log 2>&1
i=0
for group in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
  "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
  "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
  "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $group -d $O/p$i -o pmc --output-format csv -- python3 -u tools/wal_dev_probe.py 2 > $O/p$i.log 2>&1
done
