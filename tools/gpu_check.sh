#!/bin/bash
# One GPU call: the GPU test suite, then C3 bench lines (default plane, the
# bf16 plane, clustered data).  Stops at the first fault / time limit; a
# plain test failure (pytest exit 1) still lets the benches run.
# Usage (through gpurun): bash tools/gpu_check.sh <tag> [pytest -k expr|""] [ab_env specs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-chk}; K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
if [ -n "$K" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > "$OUT/tests.log" 2>&1
else
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > "$OUT/tests.log" 2>&1
fi
rc=$?; tail -5 "$OUT/tests.log"; ok $rc || { echo "tests rc=$rc: stop"; exit $rc; }
shift 2 2>/dev/null || shift $#
[ $# -gt 0 ] && exec_specs=("$@") || exec_specs=("i8:" "bf16:VS_FILTER=bf16" "cl_i8::--data clustered" "cl_bf16:VS_FILTER=bf16:--data clustered")
bash tools/ab_env.sh "$TAG" "${exec_specs[@]}"
