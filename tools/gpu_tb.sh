#!/bin/bash
# One GPU call: some GPU test files, then bench lines (tools/ab_env.sh specs).
# Stops at a fault / abort / time limit (anything but pytest's 0 or 1).
# Usage (through gpurun): bash tools/gpu_tb.sh <tag> "<test files / -k 'expr'>" [ab_env specs...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  # TESTS may hold quoted arguments (-k "a or b"): word-split by the shell
  eval "timeout -k 10 1000 python3 -u -m pytest $TESTS -m gpu -v --timeout 240 --timeout-method thread" > "$OUT/tests.log" 2>&1
  rc=$?
  tail -3 "$OUT/tests.log"
  { [ $rc -eq 0 ] || [ $rc -eq 1 ]; } || { echo "tests rc=$rc: stop"; exit $rc; }
fi
[ $# -gt 0 ] && bash tools/ab_env.sh "$TAG" "$@"
