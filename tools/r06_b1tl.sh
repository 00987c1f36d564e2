#!/bin/bash
# One batch-1 search's kernel timeline over C3's 10M rows (device outputs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06b1}
mkdir -p "$OUT"
for spec in "b1:--n 10000000 --b 1" "b1k100:--n 10000000 --b 1 --k 100"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
    -- python3 tools/step_timeline.py $args > "$OUT/$tag.log" 2>&1 || { echo "$tag failed rc=$?"; tail -5 "$OUT/$tag.log"; exit 1; }
  f=$(find "$OUT/$tag" -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py --report "$f" > "$OUT/$tag.txt" && rm -rf "$OUT/$tag"
  grep "one search" "$OUT/$tag.log"; cut -c1-100 "$OUT/$tag.txt"
done
