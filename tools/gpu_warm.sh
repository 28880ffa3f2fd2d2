# Warm-up floor check: the driver's --steps 20 --warmup 5 with a 1 s and a 3 s warm-up floor,
# alternated three times in one call (cfg2).
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/warm
mkdir -p $O
for i in 1 2 3; do
  for m in 1000 3000; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --min-warmup-ms $m --no-cpu-baseline --no-pipelined >> $O/w$m.jsonl 2>> $O/err.log
  done
done
