// Device-side helpers shared by the kernel translation units (gfx950 only).
#pragma once

#include "vs_internal.h"

namespace vs {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
#define VS_LDS(p) ((__attribute__((address_space(3))) void*)(p))

// ---------------------------------------------------------------------------
// Sorted register lists.  Entry 0 is the best.  Empty slots hold (FLT_MAX, -1):
// a candidate enters only if it is lexicographically smaller than the last
// entry, which reproduces faiss's strict admission `C::cmp(heap_top, dis)`
// against the neutral value (+/-FLT_MAX) and its id tie-break.  NaN keys never
// enter (every comparison with NaN is false), as in faiss.
template <typename IdT>
__device__ __forceinline__ bool lex_less(float ka, IdT ia, float kb, IdT ib) {
  return (ka < kb) || (ka == kb && ia < ib);
}

template <int KP, typename IdT>
__device__ __forceinline__ void list_init(float (&lk)[KP], IdT (&li)[KP]) {
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    lk[j] = FLT_MAX;
    li[j] = (IdT)-1;
  }
}

template <int KP, typename IdT>
__device__ __forceinline__ void list_insert(float (&lk)[KP], IdT (&li)[KP], float key, IdT id) {
  if (lex_less(key, id, lk[KP - 1], li[KP - 1])) {
    lk[KP - 1] = key;
    li[KP - 1] = id;
#pragma unroll
    for (int j = KP - 1; j > 0; --j) {
      const bool sw = lex_less(lk[j], li[j], lk[j - 1], li[j - 1]);
      const float a = lk[j], b = lk[j - 1];
      const IdT ia = li[j], ib = li[j - 1];
      lk[j] = sw ? b : a;
      lk[j - 1] = sw ? a : b;
      li[j] = sw ? ib : ia;
      li[j - 1] = sw ? ia : ib;
    }
  }
}

__device__ __forceinline__ float l2_from_ip(float qn, float xn, float ip) {
  // faiss exhaustive_L2sqr_blas: dis = x_norms[i] + y_norms[j] - 2 * ip; if (dis < 0) dis = 0.
  // Written without contraction so the rounding is the two-step one; NaN stays NaN.
#pragma clang fp contract(off)
  const float dis = (qn + xn) - 2.0f * ip;
  return dis < 0.0f ? 0.0f : dis;
}

__device__ __forceinline__ float wave_sum(float v) {
  v += __shfl_xor(v, 32);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

// Merges two sorted lists held in LDS (a, b) into registers (best KP of the union).
template <int KP, typename IdT>
__device__ __forceinline__ void merge2_sorted(const float* ak, const IdT* ai, const float* bk,
                                              const IdT* bi, float (&ok)[KP], IdT (&oi)[KP]) {
  int ia = 0, ib = 0;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    const float ka = ak[ia], kb = bk[ib];
    const IdT xa = ai[ia], xb = bi[ib];
    const bool ta = !lex_less(kb, xb, ka, xa);
    ok[j] = ta ? ka : kb;
    oi[j] = ta ? xa : xb;
    ia += ta ? 1 : 0;
    ib += ta ? 0 : 1;
  }
}

// The same for the first `lim` outputs only (both inputs hold at least `lim`
// written entries, padded with empty ones); outputs past lim are left as they are.
template <int KP, typename IdT>
__device__ __forceinline__ void merge2_sorted_n(const float* ak, const IdT* ai, const float* bk,
                                                const IdT* bi, float (&ok)[KP], IdT (&oi)[KP],
                                                int lim) {
  int ia = 0, ib = 0;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    if (j >= lim) break;
    const float ka = ak[ia], kb = bk[ib];
    const IdT xa = ai[ia], xb = bi[ib];
    const bool ta = !lex_less(kb, xb, ka, xa);
    ok[j] = ta ? ka : kb;
    oi[j] = ta ? xa : xb;
    ia += ta ? 1 : 0;
    ib += ta ? 0 : 1;
  }
}

}  // namespace vs
