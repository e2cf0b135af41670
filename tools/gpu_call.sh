#!/bin/bash
# Local helper (never runs on the GPU box): one gpurun call, retried only while
# the pool has no free box (exit 3: nothing ran, nothing charged).
# usage: tools/gpu_call.sh OUTDIR TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
mkdir -p "$OUT"
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT/call.log" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "no box (attempt $i), retrying in 90 s" >> "$OUT/retry.log"
  sleep 90
done
echo "done rc=$rc" >> "$OUT/call.log"
