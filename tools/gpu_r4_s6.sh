set -u
# Round-4 step 6: group-pass density thresholds (in-process A/B of builds at HEAD with other tile
# thresholds: g8x = 8-lane pass only at >= 3968 of 4096 blocks; g4b / g4c = 4-lane pass at >= 2048 /
# 3072 instead of 1024) and a kernel trace of the 300-1000 B gapped batch (CSV).
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s6
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_g8x.so tools/ab/libtkv_g8x_g4b.so tools/ab/libtkv_g8x_g4c.so --rounds 4 --reps 5 --only irregular > $O/probe_thresholds.jsonl 2>&1
rc=$?; echo "probe rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace300 -o run -- python3 $GRAFT_REPO_ROOT/tools/lane_probe.py $GRAFT_REPO_ROOT/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "300-1000 B, 8 B gaps" > $O/trace300.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
