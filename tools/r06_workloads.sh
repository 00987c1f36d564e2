#!/bin/bash
# Bench lines of the other workloads on the last build: C4 (self-join 1M,
# cosine top-50), C5 (50M bf16, batch 8, mutations), C3 with L2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06zw}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for spec in "c4:--workload c4" "c5:--workload c5" "c3l2:--metric l2"; do
  name=${spec%%:*}; args=${spec#*:}
  echo "[$(date +%T)] $name"
  timeout -k 10 600 python3 -u bench.py $args --no-cpu-baseline --wide-k-steps 0 --any-k 0 \
    --clustered-steps 0 > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "$name rc=$?"; tail -5 $OUT/bench_$name.err; exit 1; }
  python3 -c "
import json
d=json.loads([x for x in open('$OUT/bench_$name.json') if x.startswith('{')][-1])
print('$name', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'])"
done
