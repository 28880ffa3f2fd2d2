#!/bin/bash
# Profiling evidence of the current tree on one MI355X (the round's profiles/rN/final/ comes from
# this): kernel traces of the cfg2 and cfg4 bench commands (one stream, no side measurements) with
# the timed launches summarized (tools/trace_timed.py), one rocprofv3 --pmc FETCH_SIZE pass per
# config (cfg2-cfg5) of a short bench run, and FETCH passes plus a kernel trace of the device WAL
# verify on the small-record, Zipf and values-made-of-records images (tools/wal_sweep_probe.py).
# Usage: tools/gpu_evidence.sh <name>; output in gpurun_out/<name>/.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-evidence}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --no-pipelined --no-more-configs --no-paths --no-cpu-baseline --no-e2e --no-wal-payloads"
for C in cfg2 cfg4; do
  timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/trace_$C -o run --output-format csv -- python3 $B --config $C > $O/trace_$C.log 2>&1
  rc=$?; echo "trace $C rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/trace_$C.log; exit $rc; fi
done
python3 $R/tools/trace_timed.py $(find $O/trace_cfg2 -name "*kernel_trace.csv" | head -1) 'crc_packed<true>' 200 > $O/cfg2_timed.json && cat $O/cfg2_timed.json
python3 $R/tools/trace_timed.py $(find $O/trace_cfg4 -name "*kernel_trace.csv" | head -1) 'crc_stream' 200 > $O/cfg4_timed.json && cat $O/cfg4_timed.json
for C in cfg2 cfg3 cfg4 cfg5; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$C -o pmc --output-format csv -- python3 $B --config $C --steps 5 --warmup 2 --min-warmup-ms 0 > $O/pmc_$C.log 2>&1
  rc=$?; echo "pmc $C rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_$C.log; exit $rc; fi
done
for I in small zipf adv; do
  timeout -k 10 -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_wal_$I -o pmc --output-format csv -- python3 $R/tools/wal_sweep_probe.py --image $I --reps 3 > $O/pmc_wal_$I.log 2>&1
  rc=$?; echo "pmc wal $I rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_wal_$I.log; exit $rc; fi
done
timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/trace_wal -o run --output-format csv -- python3 $R/tools/wal_sweep_probe.py --image both --reps 5 > $O/trace_wal.log 2>&1
rc=$?; echo "trace wal rc=$rc"
exit $rc
