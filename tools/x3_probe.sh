#!/bin/bash
# Builds timing-only diagnostic variants of libvsearch.so next to the real one
# (results are wrong by design):  _pN = VS_X3_PROBE=N (see vs_gemm_x3.hip).
set -e
cd "$(dirname "$0")/../book-recommendation-engine_amd/csrc"
build() {  # <suffix> <defines...>
  local sfx=$1; shift
  mkdir -p build$sfx
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize "$@" -c vs_gemm_x3.hip -o build$sfx/vs_gemm_x3.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../vsearch/libvsearch$sfx.so \
    build/vs_api.o build/vs_gemm.o build$sfx/vs_gemm_x3.o build/vs_gemv.o build/vs_skinny.o build/vs_support.o
}
for p in ${PROBES:-1 2 3 4 5}; do build _p$p -DVS_X3_PROBE=$p & done
wait
