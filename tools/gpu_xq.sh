set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/explore.py --only "pp T,packed D4 I2" --rounds 6 > gpurun_out/pp_cfg2.txt 2>&1
timeout -k 10 500 python3 tools/explore.py --len 65536 --gib 16 --only "pp T,pri3 skew 0.6,packed D4 I2" --rounds 4 --reps 3 > gpurun_out/pp_cfg3.txt 2>&1
