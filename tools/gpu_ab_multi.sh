# In-process comparison of the product library with the probe builds in tools/ab/ (ab_multi.py).
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${AB_OUT:-abm}; mkdir -p $O
timeout -k 10 600 python3 tools/ab_multi.py --no-check tinykvpp_amd/libtkv_crc32.so tools/ab/*.so > $O/ab.jsonl 2> $O/ab.err
