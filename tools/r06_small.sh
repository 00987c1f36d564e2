#!/bin/bash
# Round 6: small-batch tests (the later stages skipped on host-output calls),
# host-path batch-1 latency with and without the skip (VS_SMALL_SKIP), then
# C5 with and without the plane passes' non-temporal row pieces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-sm}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "small or batch1 or skinny or b1 or test_gpu_c5 or test_gpu_bf16 or test_gpu_store or test_gpu_planes" > $OUT/tests.log 2>&1
rc=$?; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || { echo "tests rc=$rc: stop"; exit $rc; }
for v in 1 0 1 0; do
  VS_SMALL_SKIP=$v timeout -k 10 300 python3 -u tools/b1_host_latency.py >> $OUT/b1_host.jsonl 2> $OUT/b1_host.err || exit $?
done
cat $OUT/b1_host.jsonl
bash tools/r06_c5.sh $TAG
