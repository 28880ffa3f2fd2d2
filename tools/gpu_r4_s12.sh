set -u
# Round-4 step 12: the device WAL verify's walk on the 64 KiB table image with two workgroups per CU
# (tools/ab/libtkv_wal16.so) against the product, in one process (results must agree).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s12
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/ab_wal.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_wal16.so --rounds 6 > $O/ab_wal.jsonl 2>&1
rc=$?; echo "ab_wal rc=$rc"; grep "^{" $O/ab_wal.jsonl | cut -c1-260; [ $rc -eq 0 ] || exit $rc
# and the walk lookahead: list walks 3 steps ahead (list3), also the lane phase / group passes (walk3)
timeout -k 10 400 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_list3.so tools/ab/libtkv_walk3.so --rounds 4 --reps 5 --only irregular > $O/probe_ahead.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
