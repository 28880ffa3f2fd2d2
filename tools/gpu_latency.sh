set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 tools/bench_formats.py > gpurun_out/bench_formats.jsonl 2> gpurun_out/bench_formats.err
TKV_UPDATE_SMALL_BYTES=0 timeout -k 10 400 python3 tools/bench_formats.py > gpurun_out/bench_formats_nosmall.jsonl 2>> gpurun_out/bench_formats.err
