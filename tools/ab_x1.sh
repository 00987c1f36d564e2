#!/bin/bash
# Interleaved A/B of libvsearch builds on the C3 bench (run through gpurun):
#   tools/ab_x1.sh <tag> <variant>... [-- bench args]
# variant "base" = vsearch/libvsearch.so, otherwise vsearch/libvsearch_<variant>.so
# (tools/build_variant.sh); "<variant>@NAME=VAL" also sets an environment
# variable; each variant is one bench.py process, two rounds.
set -u
TAG=${1:-ab}; shift || true
VARS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VARS+=("$1"); shift; done
[ $# -gt 0 ] && shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_${TAG}
mkdir -p "$OUT"
for round in 1 2; do
  for v in "${VARS[@]}"; do
    name=${v%%@*}; envs=(); [ "$name" != "$v" ] && envs=("${v#*@}")
    lib=book-recommendation-engine_amd/vsearch/libvsearch_$name.so
    [ "$name" = base ] && lib=book-recommendation-engine_amd/vsearch/libvsearch.so
    env "${envs[@]}" VSEARCH_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 \
      --batch1-steps 0 --wide-k-steps 0 --no-cpu-baseline "$@" > "$OUT/${v}_r${round}.log" 2>&1 || { echo "$v failed"; exit 1; }
    python3 - "$OUT/${v}_r${round}.log" "$v" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[2]:10s} value={d['value']:.0f} ms/step={d['ms_per_step']:.2f} "
      f"frac={d['roofline']['frac']:.4f} {d['roofline']['per_launch'][-40:]} "
      f"fv={d.get('filter_verify', {}).get('wide_checked')}/{d.get('filter_verify', {}).get('fallback_queries')}")
PY
  done
done
