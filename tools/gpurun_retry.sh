#!/bin/bash
# Submit one gpurun command; resubmit while gpurun reports that nothing ran
# (exit 3: no box or slot; or a transient infrastructure failure before the
# command started: "status=transient", nothing charged).  Anything else ends it.
#   tools/gpurun_retry.sh <out-file> <gpurun timeout s> <command>
out=$1; lim=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then break; fi
  echo "[retry] try $i: rc=$rc, nothing ran; waiting" >> "$out.tries"
  sleep 180
done
echo "[retry] rc=$rc" >> "$out"
