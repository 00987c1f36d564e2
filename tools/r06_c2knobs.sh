#!/bin/bash
# C2 / rank knobs on the last build (interleaved): workgroup target between one
# and two rounds (VS_X1_WGS), split-pass list share (VS_X1_SPLIT).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-c2knobs}
bash tools/ab_env.sh $TAG "c2_def::--workload c2" "c2_w384:VS_X1_WGS=384:--workload c2" \
  "c2_w320:VS_X1_WGS=320:--workload c2" "c2_s16:VS_X1_SPLIT=16:--workload c2" \
  "c2_s4:VS_X1_SPLIT=4:--workload c2" "c2_def2::--workload c2" \
  "r8_def::--ntotal 1250000" "r8_w384:VS_X1_WGS=384:--ntotal 1250000" \
  "r8_w640:VS_X1_WGS=640:--ntotal 1250000" "r8_def2::--ntotal 1250000"
