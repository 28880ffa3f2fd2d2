# Native rocprofv3 --kernel-trace --stats CSV summaries of the cfg3 and cfg5 bench commands.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/native
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/native/cfg3 -o run -- python3 $R/bench.py --config cfg3 --no-cpu-baseline --no-pipelined --no-e2e > $R/gpurun_out/native/cfg3.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/native/cfg5 -o run -- python3 $R/bench.py --config cfg5 --no-cpu-baseline --no-pipelined --steps 40 --warmup 20 > $R/gpurun_out/native/cfg5.log 2>&1
