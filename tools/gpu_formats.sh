set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 tools/bench_formats.py > gpurun_out/bench_formats.jsonl 2> gpurun_out/bench_formats.err
timeout -k 10 300 python3 bench.py --config cfg5 --steps 50 --warmup 20 > gpurun_out/bench_cfg5.json 2> gpurun_out/bench_cfg5.err
