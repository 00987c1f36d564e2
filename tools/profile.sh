#!/bin/bash
# Collects the rocprofv3 evidence for bench.py on one MI355X (run through gpurun;
# the wide-k legs, whose passes have other launch sizes, left out so the trace's
# per-kernel averages are those of the line's own kernel):
#   1) --kernel-trace --stats       per-kernel durations (must agree with bench.py's HIP events)
#   2) --pmc FETCH_SIZE             HBM read traffic per dispatch (own pass)
#   3) --pmc WRITE_SIZE             HBM write traffic per dispatch (own pass)
# Usage: tools/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
ARGS=("$@")
# PMC passes: one timed search after PMC_WARMUP untimed ones (the adaptive
# plane order of clustered data settles after a few searches)
PW=${PMC_WARMUP:-0}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
  -- python3 bench.py --steps 3 --warmup 1 --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline "${ARGS[@]}" > "$OUT/bench_trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run \
  -- python3 bench.py --steps 1 --warmup "$PW" --batch1-steps 3 --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline "${ARGS[@]}" > "$OUT/bench_fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run \
  -- python3 bench.py --steps 1 --warmup "$PW" --batch1-steps 3 --wide-k-steps 0 --any-k 0 --clustered-steps 0 --no-cpu-baseline "${ARGS[@]}" > "$OUT/bench_write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
find "$OUT" -name "*.csv" | head -20
echo "profile ok"
