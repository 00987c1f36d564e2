#!/bin/bash
# A/B of the tail wait (VS_TAIL_WAIT=0 keeps every later-stage launch over an
# empty count) on C2, the 1.25M-row rank stand-in and C3, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-tail}
bash tools/ab_env.sh $TAG "c2_on::--workload c2" "c2_off:VS_TAIL_WAIT=0:--workload c2" \
  "r8_on::--ntotal 1250000" "r8_off:VS_TAIL_WAIT=0:--ntotal 1250000" \
  "c2_on2::--workload c2" "c2_off2:VS_TAIL_WAIT=0:--workload c2" \
  "c3_on::" "c3_off:VS_TAIL_WAIT=0:"
