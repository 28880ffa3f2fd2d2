#!/bin/bash
# Per-call cost of update(): GPU path vs host span path vs the reference, 28 B - 2 MiB (crossover).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 200 tools/build/put_latency oracle/_ref/libref_crc32.so > $O/put_latency.jsonl 2> $O/put_latency.err
rc=$?; echo "put_latency rc=$rc"; cat $O/put_latency.jsonl | head -12
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "side_stream or update" > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log
exit $rc
