#!/bin/bash
# FETCH_SIZE calibration of the packed kernel's load pattern (tools/fetch_calib.hip): rates, then one
# --pmc FETCH_SIZE pass and one TCC hit/miss pass, each its own run.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3cal
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/fetch_calib > $O/rates.jsonl 2>&1 || exit 1
cat $O/rates.jsonl
timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o pmc --output-format csv -- $R/tools/fetch_calib > $O/fetch.log 2>&1 || exit 1
timeout -k 10 -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc -o pmc --output-format csv -- $R/tools/fetch_calib > $O/tcc.log 2>&1 || exit 1
echo done
