#!/bin/bash
# Replay with 16-B list pieces: one-search timelines (C2, the rank), then the
# GPU suite, smoke() and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r06rp}
mkdir -p "$OUT"
for spec in "c2:--n 1000000 --b 1024" "r8:--n 1250000 --b 4096"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
    -- python3 tools/step_timeline.py $args > "$OUT/$tag.log" 2>&1 || { echo "$tag failed rc=$?"; tail -5 "$OUT/$tag.log"; exit 1; }
  f=$(find "$OUT/$tag" -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py --report "$f" > "$OUT/$tag.txt" && rm -rf "$OUT/$tag"
  grep -E "replay|span" "$OUT/$tag.txt" | cut -c1-90
done
bash tools/r06_final.sh tests ${1:-r06rp}
