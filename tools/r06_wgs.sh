#!/bin/bash
# A/B of the filter pass's workgroup target (VS_X1_WGS: 512 default = two per
# CU, 256 = one round) on the short passes: C2, the 1.25M-row rank stand-in.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-wgs}
bash tools/ab_env.sh $TAG "c2_512::--workload c2" "c2_256:VS_X1_WGS=256:--workload c2" \
  "r8_512::--ntotal 1250000" "r8_256:VS_X1_WGS=256:--ntotal 1250000" \
  "c2_512b::--workload c2" "c2_256b:VS_X1_WGS=256:--workload c2"
