set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/explore.py --only "stag,packed D4 I2" --rounds 5 > gpurun_out/stag_cfg2.txt 2>&1
timeout -k 10 300 python3 tools/explore.py --len 65536 --gib 16 --only "stag,packed D4 I2" --rounds 3 --reps 3 > gpurun_out/stag_cfg3.txt 2>&1
