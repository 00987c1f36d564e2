#!/bin/bash
# A/B of the non-temporal policy on the plane passes' row pieces (VS_SKINNY_NT):
# C3 batch 1 (skinny_plane_topk_i8 over the 15.4 GB int8 plane), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-snt}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in a b; do
  for v in 0 1; do
    VS_SKINNY_NT=$v timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --batch1-steps 40 \
      --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline > $OUT/nt$v$r.json 2> $OUT/nt$v$r.err || exit $?
    python3 -c "
import json
d=json.loads([x for x in open('$OUT/nt$v$r.json') if x.startswith('{')][-1]); b=d['batch1']
print('nt=$v $r', b['ms_per_query'], b['kernel_ms'], b.get('frac_hbm_peak'), b.get('achieved_GBs'))"
  done
done
