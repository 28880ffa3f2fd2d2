# A/B: first row loads issued before the LDS table fill ("early") vs the product order, one process each size.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 240 python3 tools/explore.py --len 4096 --gib 4 --rounds 15 --reps 5 --only "pri3" > gpurun_out/early_4k.txt 2>&1
timeout -k 10 240 python3 tools/explore.py --len 65536 --gib 16 --rounds 9 --reps 3 --only "pri3" > gpurun_out/early_64k.txt 2>&1
