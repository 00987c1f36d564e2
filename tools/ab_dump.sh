#!/bin/bash
# A/B of the filter pass's dump launches (vs_gemm_x1.hip header) against list
# launches only (VS_X1_DUMP=0), through gpurun:
#   gpurun -- bash tools/ab_dump.sh
# C3 uniform, clustered, C4 and C2, two interleaved rounds each (tools/ab_x1.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/ab_x1.sh dump_c3 base base@VS_X1_DUMP=0 || exit 1
bash tools/ab_x1.sh dump_cl base base@VS_X1_DUMP=0 -- --data clustered || exit 1
bash tools/ab_x1.sh dump_c4 base base@VS_X1_DUMP=0 -- --workload c4 || exit 1
bash tools/ab_x1.sh dump_c2 base base@VS_X1_DUMP=0 -- --workload c2 || exit 1
