set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 240 python3 tools/explore.py --only "dyn,packed D4 I2" --rounds 5 > gpurun_out/dyn_ab_4k.log 2>&1
timeout -k 10 200 python3 tools/wave_tail.py 1 > gpurun_out/dyn_tail.log 2>&1
timeout -k 10 200 python3 tools/explore.py --only "dyn D4 I2 C16,dyn D4 I2 C32,packed D4 I2" --len 65536 --rounds 3 > gpurun_out/dyn_ab_64k.log 2>&1
timeout -k 10 200 python3 tools/explore.py --only "dyn D4 I2 C16,packed D4 I2" --len 12288 --gib 3.9 --rounds 3 > gpurun_out/dyn_ab_12k.log 2>&1
timeout -k 10 200 python3 tools/explore.py --only "dyn D4 I2 C16,packed D4 I2" --len 4096 --gib 3.9 --rounds 3 > gpurun_out/dyn_ab_4k_ragged.log 2>&1
