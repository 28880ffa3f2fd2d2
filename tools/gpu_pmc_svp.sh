set -e
cd $GRAFT_REPO_ROOT
bash tools/pmc_cmd.sh $GRAFT_REPO_ROOT/gpurun_out/pmc_svp tools/stream_vs_packed.py --reps 10
