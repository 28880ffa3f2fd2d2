set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/explore.py --only "strided,stream,pat seg64 D4 fin0,pat coal D4 fin0,pat seg64 D4 fin2,packed D4 I2" --rounds 5 > gpurun_out/explore_strided.log 2>&1
