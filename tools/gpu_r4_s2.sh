set -u
# Round-4 step 2: lane-kernel PMC passes, then the record-check kernel's FETCH pass.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s2
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_lanepmc.sh r4_s2/lanepmc
rc=$?; echo "lanepmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_r4.py $O/lanepmc > $O/lanepmc_summary.txt 2>&1; tail -80 $O/lanepmc_summary.txt
# FETCH_SIZE of the record check (wal_rec_lanes) and of the generic batch on the same 36-byte payloads
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE -d $O/rec_fetch -o pmc --output-format csv -- python3 tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 3 --only "36 B" > $O/rec_fetch.log 2>&1
rc=$?; echo "rec fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/rec_sq -o pmc --output-format csv -- python3 tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 3 --only "36 B" > $O/rec_sq.log 2>&1
rc=$?; echo "rec sq rc=$rc"; exit $rc
