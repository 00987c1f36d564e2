#!/bin/bash
# Times bench.py (C3) with the diagnostic builds of tools/x3_probe.sh:
#   PROBES="6 7 8" bash tools/x3_probe_run.sh      (run through gpurun)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=book-recommendation-engine_amd/vsearch
run() { # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --batch1-steps 0 > gpurun_out/probe_$tag.log 2>&1 || { echo "$tag failed rc=$?"; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/probe_$tag.log)"
}
run base
for p in ${PROBES:-}; do run p$p VSEARCH_LIB=$PWD/$L/libvsearch_p$p.so; done
