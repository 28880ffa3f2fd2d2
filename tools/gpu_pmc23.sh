# PMC passes (one rocprofv3 --pmc run per counter group) of the cfg2 and cfg3 bench commands.
set -e
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc.sh $R/gpurun_out/pmc_cfg2 --steps 3 --warmup 3
bash $R/tools/pmc.sh $R/gpurun_out/pmc_cfg3 --config cfg3 --no-e2e --steps 3 --warmup 3
