#!/bin/bash
# Submit one gpurun command, resubmitting only while gpurun answers 3 (no box
# or slot free: nothing ran, nothing charged).  Any other exit code ends it.
#   tools/gpurun_when_free.sh <out-file> <gpurun timeout s> <command>
out=$1; lim=$2; cmd=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  echo "[when_free] try $i: no slot, waiting" >> "$out.tries"
  sleep 240
done
echo "[when_free] rc=$rc" >> "$out"
