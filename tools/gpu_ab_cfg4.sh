# cfg4 bench A/B: tools/ab/libtkv_old.so vs the current build, alternating, one box; then the
# kernel trace of the current build's cfg4 bench.
set -e
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2 3 4 5 6; do
  timeout -k 10 300 python3 tools/ab_lib.py tools/ab/libtkv_old.so bench.py --config cfg4 --no-cpu-baseline >> gpurun_out/ab_cfg4_old.jsonl 2>> gpurun_out/ab_cfg4.err
  timeout -k 10 300 python3 bench.py --config cfg4 --no-cpu-baseline >> gpurun_out/ab_cfg4_new.jsonl 2>> gpurun_out/ab_cfg4.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_cfg4 -o run -- python3 $R/bench.py --config cfg4 --no-cpu-baseline > $R/gpurun_out/prof_cfg4.log 2>&1
