# Launch time against batch size for the product partition (explorer "pri3" family), 4 KiB and
# 64 KiB blocks: separates the fixed per-launch cost from the per-byte cost.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/sweep
for len in 4096 65536; do
  for gib in 1 2 4 8 16; do
    echo "## len $len gib $gib" >> gpurun_out/sweep/sweep.txt
    timeout -k 10 120 python3 -u tools/explore.py --only "pri3" --rounds 5 --len $len --gib $gib 2>&1 | grep -v amdgpu.ids >> gpurun_out/sweep/sweep.txt
  done
done
