#!/bin/bash
# Round 5, step 12: 7 KiB regions x 12 waves; adversarial 1 GiB image; tables at LDS 0, u32 positions, buffer loads, cheaper marks: WAL tests, A/B against round 4 and the previous commit, PMC of the sweep.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s12
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_fuzz.py tests/test_gpu_formats.py -m gpu -q -k "wal or Wal" --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest_wal.log 2>&1
rc=$?; echo "pytest wal rc=$rc"; tail -2 $O/pytest_wal.log; grep -E "^FAILED|^ERROR" $O/pytest_wal.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tools/ab/libtkv_r4.so tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
timeout -k 10 200 python -u tools/wal_sweep_probe.py tools/ab/libtkv_stamp.so --reps 3 > $O/stamp.log 2>&1
echo "stamp rc=$?"; cat $O/stamp.log | grep image
timeout -k 10 300 python -u tools/wal_sweep_probe.py --reps 5 --image adv > $O/adv.log 2>&1
echo "adv rc=$?"; grep image $O/adv.log
cd /tmp && export TMPDIR=/tmp
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $g -d $O/pmc_$i -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 2 --image small > $O/pmc_$i.log 2>&1
  echo "pmc $i rc=$?"
done
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py --reps 4 > $O/trace.log 2>&1
echo "trace rc=$?"; grep image $O/trace.log
echo done
