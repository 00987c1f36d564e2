#!/bin/bash
# The 1.25M-row rank stand-in (153 tiles per workgroup): five 32-tile launches
# (default) vs a split pass (list launch over 1/den of the tiles, one dump
# launch over the rest) via VS_X1_CHUNK_TILES, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rankchunk}
bash tools/ab_env.sh $TAG "r8_def::--ntotal 1250000" "r8_c64:VS_X1_CHUNK_TILES=64:--ntotal 1250000" \
  "r8_c160:VS_X1_CHUNK_TILES=160:--ntotal 1250000" \
  "r8_c64s16:VS_X1_CHUNK_TILES=64 VS_X1_SPLIT=16:--ntotal 1250000" \
  "r8_c64s4:VS_X1_CHUNK_TILES=64 VS_X1_SPLIT=4:--ntotal 1250000" \
  "r8_def2::--ntotal 1250000" "r8_c64b:VS_X1_CHUNK_TILES=64:--ntotal 1250000" \
  "r8_c40:VS_X1_CHUNK_TILES=40:--ntotal 1250000"
