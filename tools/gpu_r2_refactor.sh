# Round-2 check after moving the explorer-only variants out of the product header: GPU parity suite,
# smoke, and an in-process A/B of the previous build (tools/ab/libtkv_old.so) against this one.
set -e
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r2_refactor
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 tools/ab_libs.py tools/ab/libtkv_old.so tinykvpp_amd/libtkv_crc32.so > $O/ab.jsonl 2> $O/ab.err
