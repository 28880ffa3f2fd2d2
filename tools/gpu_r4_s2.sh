set -u
# Round-4 step 2: lane-kernel PMC passes, then the record-check kernel's FETCH pass.
O=$GRAFT_REPO_ROOT/gpurun_out/r4_s2
mkdir -p $O
cd $GRAFT_REPO_ROOT
bash tools/gpu_r4_lanepmc.sh r4_s2/lanepmc
rc=$?; echo "lanepmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_r4.py $O/lanepmc > $O/lanepmc_summary.txt 2>&1; tail -80 $O/lanepmc_summary.txt
