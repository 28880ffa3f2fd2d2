#!/bin/bash
# Round 5, step 19: crc_list_lanes (one pass over (offset, length) for irregular batches of lane
# blocks, the general path gated on it): tests, then A/B against HEAD (prev) in one process.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5s25
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_fuzz.py tests/test_gpu_formats.py tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_wal_device.py -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 4 > $O/lane_probe.jsonl 2>&1
echo "lane rc=$?"; grep irregular $O/lane_probe.jsonl | cut -c1-170
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_prev.so --rounds 3 > $O/rec_probe.jsonl 2>&1
echo "rec rc=$?"; grep batch_device $O/rec_probe.jsonl | cut -c1-200
timeout -k 10 300 python -u tools/ab_lib.py tools/ab/libtkv_prev.so bench.py --config cfg4 --no-cpu-baseline --no-pipelined --no-more-configs --steps 50 --warmup 20 > $O/cfg4_prev.json 2>&1
timeout -k 10 300 python -u bench.py --config cfg4 --no-cpu-baseline --no-pipelined --no-more-configs --steps 50 --warmup 20 > $O/cfg4_new.json 2>&1
echo "cfg4 rc=$?"; tail -c 300 $O/cfg4_prev.json; echo; tail -c 300 $O/cfg4_new.json
echo done
