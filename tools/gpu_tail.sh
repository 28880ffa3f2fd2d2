# Pooled-tail variants (static share with the product priority + per-XCD chunk pools) vs the product.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/chunks
timeout -k 10 240 python3 -u tools/explore.py --only "pri3,chunks" --rounds 7 > gpurun_out/chunks/cfg2.txt 2>&1
timeout -k 10 300 python3 -u tools/explore.py --only "pri3,chunks" --rounds 5 --len 65536 --gib 16 > gpurun_out/chunks/cfg3.txt 2>&1
