#!/bin/bash
# Kernel timelines of one search (C2, the 1.25M-row rank) with the wide
# check at four rows per wave step (default) and two (VS_WIDE_ROWS=2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl2}
mkdir -p "$OUT"
for spec in "c2:--n 1000000 --b 1024" "r8:--n 1250000 --b 4096"; do
  for wr in 4 2; do
    tag=${spec%%:*}_w$wr; args=${spec#*:}
    VS_WIDE_ROWS=$wr timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
      -- python3 tools/step_timeline.py $args > "$OUT/$tag.log" 2>&1 || { echo "$tag failed rc=$?"; tail -5 "$OUT/$tag.log"; exit 1; }
    f=$(find "$OUT/$tag" -name "*kernel_trace.csv" | head -1)
    python3 tools/step_timeline.py --report "$f" | grep -v "^W2026\|^E2026" > "$OUT/$tag.txt" && rm -rf "$OUT/$tag"
    echo "$tag: $(grep 'one search' "$OUT/$tag.log") | $(tail -1 "$OUT/$tag.txt")"
    grep -E "verify|select_heads|merge_lists" "$OUT/$tag.txt" | head -6 | cut -c1-90
  done
done
