set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/explore.py --only "packed D4 I2,packed rot,stream" --rounds 7 > gpurun_out/explore_rot_4k.log 2>&1
timeout -k 10 300 python3 tools/explore.py --only "packed D4 I2,packed rot,stream" --len 65536 --rounds 5 > gpurun_out/explore_rot_64k.log 2>&1
timeout -k 10 300 python3 tools/explore.py --only "packed D4 I2,packed rot" --len 4096 --gib 3.9 --rounds 3 > gpurun_out/explore_rot_ragged.log 2>&1
