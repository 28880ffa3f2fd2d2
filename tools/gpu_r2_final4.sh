# End-of-session check of the round-2 tree on one MI355X: full GPU parity suite (incl. the randomized
# sweep), smoke, the default bench line under the kernel trace, cfg3/cfg4/cfg5 lines, the formats
# bench (WAL / SSTable rows with the reference's CPU path beside them), and a FETCH_SIZE pass of the
# default bench command (roofline.traffic).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${FINAL_OUT:-final4}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_cfg2 -o run --output-format csv -- python3 bench.py > $O/bench_cfg2.json 2> $O/bench_cfg2.err
timeout -k 10 300 python3 bench.py --config cfg3 > $O/bench_cfg3.json 2> $O/bench_cfg3.err
timeout -k 10 300 python3 bench.py --config cfg4 > $O/bench_cfg4.json 2> $O/bench_cfg4.err
timeout -k 10 400 python3 bench.py --config cfg5 --steps 50 --warmup 20 > $O/bench_cfg5.json 2> $O/bench_cfg5.err
timeout -k 10 400 python3 tools/bench_formats.py > $O/bench_formats.jsonl 2> $O/bench_formats.err
mkdir -p $O/pmc_cfg2
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_cfg2/FETCH_SIZE -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-pipelined --steps 3 --warmup 3 --min-warmup-ms 0 > $O/pmc_cfg2/FETCH_SIZE.log 2>&1
