set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 250 python3 tools/explore.py --only "skew 0.6,prio,packed D4 I2" --rounds 9 > gpurun_out/prio2_cfg2.txt 2>&1
timeout -k 10 400 python3 tools/explore.py --len 65536 --gib 16 --only "skew 0.6,prio,packed D4 I2" --rounds 6 --reps 3 > gpurun_out/prio2_cfg3.txt 2>&1
