# Pooled-tail variants (static share with the product priority + per-XCD chunk pools) vs the product.
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lean
timeout -k 10 240 python3 -u tools/explore.py --only "pri3,lean" --rounds 7 > gpurun_out/lean/cfg2.txt 2>&1
timeout -k 10 300 python3 -u tools/explore.py --only "pri3,lean" --rounds 5 --len 65536 --gib 16 > gpurun_out/lean/cfg3.txt 2>&1
