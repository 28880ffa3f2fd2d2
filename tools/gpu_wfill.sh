# Round-end rehearsal (tools/gpu_validate.sh) plus the wide table-fill A/B (explorer, one process per config).
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_validate.sh
mkdir -p gpurun_out/wfill
timeout -k 10 240 python3 -u tools/explore.py --only "pri3" --rounds 9 > gpurun_out/wfill/cfg2.txt 2>&1
timeout -k 10 300 python3 -u tools/explore.py --only "pri3" --rounds 7 --len 65536 --gib 16 > gpurun_out/wfill/cfg3.txt 2>&1
