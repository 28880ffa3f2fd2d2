set -u
# Round-4 step 13: the record check on true 44-byte records (36-byte payloads) and the 36-byte records
# the earlier probes used, then one FETCH_SIZE pass over the same probe (record-check kernels by window).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s13
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/rec_probe.py tinykvpp_amd/libtkv_crc32.so --rounds 5 --reps 5 > $O/rec_probe.jsonl 2>&1
rc=$?; echo "rec rc=$rc"; grep "^{" $O/rec_probe.jsonl | cut -c1-250; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/rec_probe.py $GRAFT_REPO_ROOT/tinykvpp_amd/libtkv_crc32.so --rounds 1 --reps 2 > $O/pmc_fetch.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
