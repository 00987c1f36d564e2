#!/bin/bash
# Round 6: GPU tests of the exact-key pages (IP k > 32 last stage) and the
# wide-k / dump / parity suites, then the workgroup target at the boundary
# batch sizes (4, 8 and 1 query tiles; default vs the other setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-t6}
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
  -k "test_gpu_wide_k or test_gpu_dump or test_gpu_parity or test_gpu_bf16" > $OUT/tests.log 2>&1
rc=$?; tail -4 $OUT/tests.log
{ [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "tests rc=$rc: stop"; exit $rc; }
bash tools/ab_env.sh $TAG "c2::--workload c2" "c2_512:VS_X1_WGS=512:--workload c2" \
  "b2048::--batch 2048" "b2048_512:VS_X1_WGS=512:--batch 2048" \
  "b256::--batch 256" "b256_512:VS_X1_WGS=512:--batch 256" "c3::"
