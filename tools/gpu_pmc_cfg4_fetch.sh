# FETCH_SIZE pass (roofline.traffic source) of the cfg4 bench command on the current prepass.
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmc4/p3 -o pmc --output-format csv -- python3 $R/bench.py --config cfg4 --no-cpu-baseline --no-pipelined --steps 50 --warmup 20 > $R/gpurun_out/pmc4/p3.log 2>&1
