#!/bin/bash
# A/B of the x1 filter pipeline forms on the C3 bench (run through gpurun):
#   tools/ab_x1.sh <tag> [bench args...]
# Each variant is one bench.py process (VS_X1_PIPE=2|4|5), interleaved twice.
set -u
TAG=${1:-ab}; shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_${TAG}
mkdir -p "$OUT"
for round in 1 2; do
  for p in ${PIPES:-2 4 5}; do
    VS_X1_PIPE=$p timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --batch1-steps 0 \
      --no-cpu-baseline "$@" > "$OUT/pipe${p}_r${round}.log" 2>&1 || { echo "pipe $p failed"; exit 1; }
    python3 - "$OUT/pipe${p}_r${round}.log" "$p" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"pipe={sys.argv[2]} value={d['value']:.0f} ms/step={d['ms_per_step']:.2f} "
      f"frac={d['roofline']['frac']:.4f} {d['roofline']['per_launch'][-60:]} "
      f"fv={d.get('filter_verify', {}).get('wide_checked')}/{d.get('filter_verify', {}).get('fallback_queries')}")
PY
  done
done
