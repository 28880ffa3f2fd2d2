#!/bin/bash
# (tools/gpu_wait.sh CMD OUT [TIMEOUT]: run in the background while working on the CPU)
# retry a gpurun call only while the pool has no box (status=transient: nothing ran, nothing charged)
CMD="$1"; OUT="$2"; TMO="${3:-900}"
for i in $(seq 1 30); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout $TMO -- "$CMD" > "$OUT" 2>&1
  if grep -q "status=transient" "$OUT"; then sleep 90; continue; fi
  break
done
echo "attempts=$i" >> "$OUT"
