#!/bin/bash
# Round 5, step 42: the tile-sum scan (rows_scan_tiles, batches of more than 128 tiles) by wave-level
# scans instead of a workgroup-wide Hillis-Steele: tests, then the irregular probe and cfg A/B against
# the build before (one process), and a kernel trace of the 100-200-byte batch.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s42
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_stream.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u tools/lane_probe.py tools/ab/libtkv_base.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --only "irregular" > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"
timeout -k 10 200 python -u tools/ab_multi.py tools/ab/libtkv_base.so tinykvpp_amd/libtkv_crc32.so --rounds 6 > $O/ab_multi.jsonl 2>&1
echo "multi rc=$?"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/t2 -o run --output-format csv -- python3 -u $R/tools/lane_probe.py $R/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 5 --only "payloads 100-200 B" > $O/t2.log 2>&1
echo "trace rc=$?"
echo done
