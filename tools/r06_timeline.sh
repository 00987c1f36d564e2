#!/bin/bash
# One search's kernel timeline for the short passes (C2: 1M rows, batch 1024;
# the 1.25M-row rank stand-in, batch 4096) and C3, from rocprofv3 kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tl}
mkdir -p "$OUT"
for spec in "c2:--n 1000000 --b 1024" "r8:--n 1250000 --b 4096" "c3:--n 10000000 --b 4096"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
    -- python3 tools/step_timeline.py $args > "$OUT/$tag.log" 2>&1 || { echo "$tag failed rc=$?"; exit 1; }
  f=$(find "$OUT/$tag" -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py --report "$f" >> "$OUT/$tag.log" && rm -rf "$OUT/$tag"
  tail -2 "$OUT/$tag.log"
done
