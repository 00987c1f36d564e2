#!/bin/bash
# A/B of the LDS-DMA cache policy on gemm_dump_s5 (VS_X1_S5=1): default, nt on
# the database pieces, nt on both; the default dump form for reference.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/ab_env.sh ${1:-nt} "s5:VS_X1_S5=1" "s5nt1:VS_X1_S5=1 VS_X1_NT=1" "s5nt3:VS_X1_S5=1 VS_X1_NT=3" "s0:VS_X1_S5=0" "s5nt1b:VS_X1_S5=1 VS_X1_NT=1"
