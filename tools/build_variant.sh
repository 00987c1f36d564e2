#!/bin/bash
# Builds an A/B variant of libvsearch.so with extra -D flags on vs_gemm_x1.hip:
#   tools/build_variant.sh <suffix> [-DNAME=VAL ...]  ->  vsearch/libvsearch_<suffix>.so
#   X1_SRC=<file> tools/build_variant.sh <suffix> ...  (another vs_gemm_x1.hip, e.g.
#   `git show HEAD~1:...` saved to a file, for before/after A/B)
# Select it at run time with VSEARCH_LIB=<that path> (tools/ab_x1.sh, x1_probe.sh).
# Needs the default build's objects (make first).
set -e
cd "$(dirname "$0")/../book-recommendation-engine_amd/csrc"
sfx=$1; shift
src=${X1_SRC:-vs_gemm_x1.hip}
mkdir -p build_$sfx
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -I. "$@" \
  -Rpass-analysis=kernel-resource-usage -x hip -c "$src" -o build_$sfx/vs_gemm_x1.o \
  2> build_$sfx/vs_gemm_x1.remarks
python3 ../../tools/check_no_spill.py build_$sfx/vs_gemm_x1.remarks gemm_topk_x1 || [ -n "${ALLOW_SPILL:-}" ]  # stamp builds: bf16 kernels spill (diagnose int8 only)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../vsearch/libvsearch_$sfx.so \
  build/vs_api.o build/vs_exact.o build/vs_gemm.o build_$sfx/vs_gemm_x1.o build/vs_gemv.o build/vs_skinny.o build/vs_support.o
echo "built vsearch/libvsearch_$sfx.so"
