#!/bin/bash
# Exact-key pages with 1,024-slot windows: the wide-k / dump tests, then the
# any-k leg of the bench (k = 100 at B = 4096 and 1) beside the default line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-xp}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "test_gpu_wide_k or test_gpu_dump" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
timeout -k 10 600 python3 -u bench.py --steps 5 --no-cpu-baseline --batch1-steps 5 --wide-k-steps 0 \
  --clustered-steps 0 > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 -c "
import json
d=json.loads([x for x in open('$OUT/bench.json') if x.startswith('{')][-1])
print(d['value'], d['ms_per_step'], [(a['k'], a['batch'], a['ms_per_search']) for a in d['any_k']])"
