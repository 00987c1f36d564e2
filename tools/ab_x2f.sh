#!/bin/bash
# A/B of the filter pass variants on one MI355X (run through gpurun):
# parity of the bf16x2v tests for each database source, then the C3 bench per
# variant.  Usage: tools/ab_x2f.sh <tag> [variant ...], variant = ENV=VAL[,ENV=VAL]
set -u
TAG=${1:-ab}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_${TAG}
mkdir -p "$OUT"
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=("VS_X2F_SRC=blocked" "VS_X2F_SRC=planes")
name() { local n=${1##*/}; n=${n//[=,.]/_}; echo "$n"; }  # log name of a variant
if [ -z "${AB_SKIP_TESTS:-}" ]; then
  for v in "${VARIANTS[@]}"; do
    n=$(name "$v")
    env ${v//,/ } timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
      -m gpu tests/test_gpu_parity.py -k "${AB_TESTS:-bf16x2v or blocked_rows}" > "$OUT/test_$n.log" 2>&1 \
      || { echo "tests failed for $v"; tail -30 "$OUT/test_$n.log"; exit 1; }
    tail -2 "$OUT/test_$n.log"
  done
fi
for v in "${VARIANTS[@]}"; do
  n=$(name "$v")
  env ${v//,/ } timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --batch1-steps 0 \
    --no-cpu-baseline > "$OUT/bench_$n.log" 2>&1 || { echo "bench failed for $v"; tail -20 "$OUT/bench_$n.log"; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' "$OUT/bench_$n.log" | head -1) $(grep -o '"frac": [0-9.]*' "$OUT/bench_$n.log" | head -1) $(grep -o '"fallback_queries": [0-9]*' "$OUT/bench_$n.log") $(grep -o '"rows_with_id_mismatch": [0-9]*' "$OUT/bench_$n.log")"
done
