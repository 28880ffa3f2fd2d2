# Native rocprofv3 --kernel-trace --stats CSV summary of the default bench command (cfg2).
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/native
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/native/cfg2 -o run -- python3 $R/bench.py --no-cpu-baseline --no-pipelined > $R/gpurun_out/native/cfg2.log 2>&1
