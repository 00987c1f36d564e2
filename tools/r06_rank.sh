#!/bin/bash
# The 1.25M-row rank of an 8-GPU C3 (one GPU standing in): default (five
# 32-tile launches: one list + four dumps) vs a split pass (list launch over
# 1/8 of each workgroup's tiles, one dump launch over the rest, one replay),
# reached through longer launches (VS_X1_CHUNK_TILES=64: three chunks, a split pass).  Two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rank}
bash tools/ab_env.sh $TAG "d1::--ntotal 1250000" "s64:VS_X1_CHUNK_TILES=64:--ntotal 1250000" \
  "d2::--ntotal 1250000" \
  "s64b:VS_X1_CHUNK_TILES=64:--ntotal 1250000"
