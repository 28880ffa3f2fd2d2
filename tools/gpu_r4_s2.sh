set -u
# Round-4 step 2: the fixed LDS-walk pass and group passes (tests + A/B), lane-kernel PMC passes (VERDICT
# r3 item 4), the record-check kernel's FETCH and SQ passes.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s2
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_wal_device.py tests/test_gpu_wal_records.py tests/test_gpu_lanes.py tests/test_gpu_fuzz.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; grep -E "^FAILED|^ERROR" $O/pytest.log | head -30
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so:walk=0 tinykvpp_amd/libtkv_crc32.so:walk=1 --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep -v amdgpu $O/ab_wal.jsonl | cut -c1-250; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lane_probe.py tools/ab/libtkv_r4base.so tinykvpp_amd/libtkv_crc32.so --rounds 3 --reps 5 --only irregular > $O/probe_irregular.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r4_lanepmc.sh r4_s2/lanepmc
rc=$?; echo "lanepmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_r4.py $O/lanepmc > $O/lanepmc_summary.txt 2>&1; tail -100 $O/lanepmc_summary.txt
# FETCH_SIZE and SQ counters of the record check (wal_rec_lanes) and the generic batch on the 36-byte payloads
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE -d $O/rec_fetch -o pmc --output-format csv -- python3 tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 3 --only "36 B" > $O/rec_fetch.log 2>&1
rc=$?; echo "rec fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/rec_sq -o pmc --output-format csv -- python3 tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 3 --only "36 B" > $O/rec_sq.log 2>&1
rc=$?; echo "rec sq rc=$rc"; exit $rc
