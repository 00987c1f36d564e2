#!/bin/bash
# C4 (1M x 1536 cosine self-join, top-50): lane lists per student 128 (default)
# vs 256 (VS_X1_SPLIT_MULT=2), two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-c4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in a b; do
  for m in 1 2; do
    VS_X1_SPLIT_MULT=$m timeout -k 10 600 python3 -u bench.py --workload c4 --no-cpu-baseline \
      > $OUT/c4_m$m$r.json 2> $OUT/c4_m$m$r.err || exit $?
    python3 -c "
import json
d=json.loads([x for x in open('$OUT/c4_m$m$r.json') if x.startswith('{')][-1]); f=d.get('filter_verify') or {}
print('mult=$m $r', d['value'], d['ms_per_step'], d['roofline']['frac'], f.get('wide_set_mean'), f.get('to_bf16_stage'), f.get('students'))"
  done
done
