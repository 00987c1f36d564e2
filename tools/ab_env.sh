#!/bin/bash
# C3 bench lines under several environment settings (through gpurun):
#   tools/ab_env.sh <tag> "<name>:<VAR=VAL ...>[:<bench args>]" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; envs=${rest%%:*}; args=""
  [ "$rest" != "$envs" ] && args=${rest#*:}
  env $envs timeout -k 10 300 python3 -u bench.py --steps 4 --warmup 1 --no-cpu-baseline \
    --batch1-steps 0 --wide-k-steps 0 --any-k 0 --clustered-steps 0 $args > "$OUT/$name.log" 2>&1
  rc=$?
  grep '^{' "$OUT/$name.log" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); r=d['roofline']; f=d.get('filter_verify') or {}
    print('$name', round(d['value']), d['ms_per_step'], r['frac'], r['per_launch'][-45:], f.get('plane'), f.get('wide_checked'), f.get('fallback_queries', f.get('fallback_students')), (f.get('exact_check') or {}).get('rows_beyond_tie_tolerance'), 'dump', (f.get('dump_launches') or {}).get('rows_dumped'), (f.get('dump_launches') or {}).get('lists_out_of_slots'), 'whole', (r.get('whole_pass') or {}).get('frac'))"
  [ $rc -eq 0 ] || { echo "$name rc=$rc: stop"; tail -5 "$OUT/$name.log"; exit $rc; }
done
