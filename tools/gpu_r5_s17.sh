#!/bin/bash
# Round 5, step 17: conflict-free lookup order in every 16-replica kernel (record check, LDS-staged
# lanes, WAL sweep); fix-up task policy (first boundary prunes, far-jump boundaries wait); regions
# inside one record passed over. Tests, then A/B against HEAD (prev) in one process.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s17
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_fuzz.py tests/test_gpu_lanes.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u tools/wal_sweep_probe.py --reps 3 --image adv > $O/adv.log 2>&1
echo "adv rc=$?"; grep image $O/adv.log | tail -3
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/ab_wal.jsonl 2>&1
echo "ab rc=$?"; grep image $O/ab_wal.jsonl
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"; tail -40 $O/lane_probe.jsonl
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/rec_probe.jsonl 2>&1
echo "rec rc=$?"; tail -12 $O/rec_probe.jsonl
echo done
