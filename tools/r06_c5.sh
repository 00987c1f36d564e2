#!/bin/bash
# C5 (50M x 1536 bf16, batch 8, 1 % removals + 1 % appends every 10 batches)
# with the plane passes' non-temporal row pieces (default) and without.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-c5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in 1 0; do
  VS_SKINNY_NT=$v timeout -k 10 900 python3 -u bench.py --workload c5 --no-cpu-baseline \
    > $OUT/c5_nt$v.json 2> $OUT/c5_nt$v.err || exit $?
  python3 -c "
import json
d=json.loads([x for x in open('$OUT/c5_nt$v.json') if x.startswith('{')][-1])
print('nt=$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['per_launch'][-60:], (d.get('recall') or d.get('recall_at_k')))"
done
