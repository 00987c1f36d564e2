#!/bin/bash
# Round-6 last build: the rank's launch length A/B (40-tile default vs 32),
# then the GPU suite, smoke() and the default bench line (tools/r06_final.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06z}
bash tools/ab_env.sh ${TAG}ab "r8_40::--ntotal 1250000" "r8_32:VS_X1_CHUNK_TILES=32:--ntotal 1250000" \
  "r8_40b::--ntotal 1250000" "r8_32b:VS_X1_CHUNK_TILES=32:--ntotal 1250000" && \
bash tools/r06_final.sh tests $TAG
