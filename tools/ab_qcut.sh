#!/bin/bash
# Pending A/B of the query cuts (DESIGN.md §3 "Query cuts"), run through gpurun:
#   bash tools/build_variant.sh qcut -DVS_X1_QCUT_K=1
#   bash tools/build_variant.sh qcutrow -DVS_X1_QCUT_K=1 -DVS_X1_ROWLOOP=1
#   gpurun -- bash tools/ab_qcut.sh
# The GPU suite on the cut build first (a failure stops here), then C3 uniform,
# clustered, C4 and C2 against the default build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/book-recommendation-engine_amd/vsearch
mkdir -p gpurun_out/ab_qcut
VS_X1_QCUT=1 VSEARCH_LIB=$L/libvsearch_qcut.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q \
  --timeout 120 --timeout-method thread > gpurun_out/ab_qcut/tests.log 2>&1 \
  || { echo "tests rc=$?"; tail -40 gpurun_out/ab_qcut/tests.log; exit 1; }
tail -2 gpurun_out/ab_qcut/tests.log
bash tools/ab_x1.sh qcut_c3 base qcut@VS_X1_QCUT=1 qcutrow@VS_X1_QCUT=1 || exit 1
bash tools/ab_x1.sh qcut_cl base qcut@VS_X1_QCUT=1 -- --data clustered || exit 1
bash tools/ab_x1.sh qcut_c4 base qcut@VS_X1_QCUT=1 -- --workload c4 || exit 1
bash tools/ab_x1.sh qcut_c2 base qcut@VS_X1_QCUT=1 -- --workload c2 || exit 1
