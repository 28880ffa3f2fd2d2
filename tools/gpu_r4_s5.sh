set -u
# Round-4 step 5: dword-by-dword lane kernel (TKV_LANES_DIRECT=2: dword- and byte-aligned blocks) against
# HEAD~1's build (tools/ab/libtkv_r4c.so); the group passes against listing every small block
# (tools/ab/libtkv_nog8.so: no 8-lane pass, libtkv_nog.so: neither pass); a kernel trace of 300-1000 B.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s5
mkdir -p $O
cd $GRAFT_REPO_ROOT
TKV_LANES_DIRECT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_lanes.py tests/test_gpu_parity.py -q --maxfail=30 --timeout 120 --timeout-method thread > $O/pytest_direct2.log 2>&1
rc=$?; echo "pytest direct2 rc=$rc"; tail -2 $O/pytest_direct2.log; grep -E "^FAILED|^ERROR" $O/pytest_direct2.log | head -30
[ $rc -le 1 ] || exit $rc
TKV_LANES_DIRECT=2 timeout -k 10 400 python -u tools/lane_probe.py tools/ab/libtkv_r4c.so tinykvpp_amd/libtkv_crc32.so --rounds 4 --reps 5 --only uniform > $O/probe_uniform_direct2.jsonl 2>&1
rc=$?; echo "probe uniform rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/lane_probe.py tinykvpp_amd/libtkv_crc32.so tools/ab/libtkv_nog8.so tools/ab/libtkv_nog.so --rounds 4 --reps 5 --only irregular > $O/probe_groups.jsonl 2>&1
rc=$?; echo "probe groups rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace300 -o run -- python3 $GRAFT_REPO_ROOT/tools/lane_probe.py $GRAFT_REPO_ROOT/tinykvpp_amd/libtkv_crc32.so --rounds 2 --reps 3 --only "300-1000 B, 8 B gaps" > $O/trace300.log 2>&1
rc=$?; echo "trace rc=$rc"; exit $rc
