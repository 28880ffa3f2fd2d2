# Wider randomized parity sweep (not part of the round-end suite): the committed fuzz cases re-seeded
# at other offsets (TKV_FUZZ_OFFSET), one pytest process per offset, stopping at the first failure.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${FUZZ_OUT:-fuzzwide}
mkdir -p $O
for off in ${FUZZ_OFFSETS:-100000 200000 300000 400000 500000 600000 700000 800000}; do
  TKV_FUZZ_OFFSET=$off timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/fuzz_$off.log 2>&1
  tail -1 $O/fuzz_$off.log
done
