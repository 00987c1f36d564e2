#!/bin/bash
# (1) the heads select's parity test; (2) C2 with the heads select vs the list
# merge; (3) the 1.25M-row rank stand-in (153 tiles per workgroup): five
# 32-tile launches (default) vs a split pass (list launch over 1/den of the
# tiles, one dump launch over the rest) via VS_X1_CHUNK_TILES, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-rankchunk}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "select_heads" -x -v --timeout 120 \
  --timeout-method thread > gpurun_out/$TAG/test_heads.log 2>&1 || { echo "heads test failed rc=$?"; tail -30 gpurun_out/$TAG/test_heads.log; exit 1; }
tail -2 gpurun_out/$TAG/test_heads.log
bash tools/ab_env.sh $TAG "c2_h1::--workload c2" "c2_h0:VS_SELECT_HEADS=0:--workload c2" \
  "r8_def::--ntotal 1250000" "r8_c64:VS_X1_CHUNK_TILES=64:--ntotal 1250000" \
  "r8_c160:VS_X1_CHUNK_TILES=160:--ntotal 1250000" \
  "c2_h1b::--workload c2" "c2_h0b:VS_SELECT_HEADS=0:--workload c2" \
  "r8_def2::--ntotal 1250000" "r8_c64b:VS_X1_CHUNK_TILES=64:--ntotal 1250000" \
  "r8_c40:VS_X1_CHUNK_TILES=40:--ntotal 1250000" && \
bash tools/r06_tl2.sh tl2
