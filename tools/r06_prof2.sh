#!/bin/bash
# Final-build rocprof evidence: C3 trace (with the batch-1 leg: the non-temporal
# skinny pass) + FETCH/WRITE PMC passes; C5 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06n}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 bash tools/profile.sh ${TAG}c3 > $OUT/prof_c3.txt 2>&1 || { echo "c3 profile rc=$?"; tail -5 $OUT/prof_c3.txt; exit 1; }
tail -2 $OUT/prof_c3.txt
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}c5 -o run \
  -- python3 bench.py --workload c5 --no-cpu-baseline > $OUT/c5_trace.log 2>&1 || { echo "c5 trace rc=$?"; exit 1; }
grep '^{' $OUT/c5_trace.log | tail -1 | cut -c1-300
