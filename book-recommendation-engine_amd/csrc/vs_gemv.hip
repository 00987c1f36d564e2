// vs_gemv.hip — streaming distance + top-k kernel for small query batches (nq <= 8).
#include "vs_device.h"

namespace vs {

// ---------------------------------------------------------------------------
// GEMV path (nq <= 8): each wave streams 4 rows at a time; lane l reads float4
// chunks l, l+64, ... of every row (1 KiB per wave instruction, fully
// coalesced), the queries sit in LDS, partial sums are reduced across the wave,
// and lane q keeps query q's list.  MODE_L2D computes sum (x-q)^2 directly, as
// faiss does for nq < 20 (fvec_L2sqr); MODE_IP the plain dot product.  Rows are
// fp32 or bf16 (widened in registers); a 16-B chunk is 4 or 8 elements.
template <typename T>
__device__ __forceinline__ void widen_chunk(const uint4 v, float (&f)[16 / sizeof(T)]) {
  if constexpr (sizeof(T) == 4) {
    f[0] = __uint_as_float(v.x);
    f[1] = __uint_as_float(v.y);
    f[2] = __uint_as_float(v.z);
    f[3] = __uint_as_float(v.w);
  } else {
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(u[i] << 16);
      f[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
    }
  }
}

// FLOOR: query q's list admits only rows strictly after (fkey[q], fid[q]) in
// (key, row) order (page p + 1 of the paged engine, vs_api.hip run_paged; a
// query with nothing left to page gets the floor (+inf, INT_MAX) and an empty
// list); `run` (optional device flag): nothing to do when *run == 0.
template <int NQ, int KP, int MODE, typename T, bool FLOOR = false>
__global__ __launch_bounds__(256) void gemv_topk(const T* __restrict__ X,
                                                 const float* __restrict__ Q, int64_t ld,
                                                 int ntotal, int rows_per_block,
                                                 float* __restrict__ pkey,
                                                 int* __restrict__ pid,
                                                 const float* __restrict__ fkey,
                                                 const int* __restrict__ fid,
                                                 const int* __restrict__ run) {
  constexpr int EPC = 16 / sizeof(T);  // elements per 16-B chunk
  extern __shared__ __attribute__((aligned(16))) float sq[];  // [NQ][ld]
  if (run && *run == 0) return;  // uniform
  const int tid = threadIdx.x;
  for (int64_t i = (int64_t)tid * 4; i < (int64_t)NQ * ld; i += 1024)
    *(f32x4*)(sq + i) = *(const f32x4*)(Q + i);
  __syncthreads();

  const int lane = tid & 63;
  const int w = tid >> 6;
  const int cpr = (int)(ld / EPC);  // chunks per row
  const int rb0 = blockIdx.x * rows_per_block;
  const int ntot16 = (ntotal + 15) & ~15;
  const int rb1 = min(rb0 + rows_per_block, ntot16);

  float lk[KP];
  int li[KP];
  list_init<KP, int>(lk, li);
  float fk = 0.0f;
  int fi = 0;
  if constexpr (FLOOR) {
    const int ql = (tid & 63) < NQ ? (tid & 63) : 0;
    fk = fkey[ql];
    fi = fid[ql];
  }

  for (int r = rb0 + 4 * w; r < rb1; r += 16) {
    float acc[4][NQ];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[a][q] = 0.0f;

    const T* xr = X + (int64_t)r * ld;
    for (int c = lane; c < cpr; c += 64) {
      uint4 xv[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = __builtin_nontemporal_load((const u32x4*)(xr + a * ld) + c);
        xv[a] = make_uint4(v.x, v.y, v.z, v.w);
      }
      float xf[4][EPC];
#pragma unroll
      for (int a = 0; a < 4; ++a) widen_chunk<T>(xv[a], xf[a]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        float qf[EPC];
#pragma unroll
        for (int e = 0; e < EPC; e += 4) {
          const f32x4 qv = *(const f32x4*)(sq + q * ld + c * EPC + e);
          qf[e] = qv.x;
          qf[e + 1] = qv.y;
          qf[e + 2] = qv.z;
          qf[e + 3] = qv.w;
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          float sacc = 0.0f;
#pragma unroll
          for (int e = 0; e < EPC; ++e) {
            if constexpr (MODE == MODE_L2D) {
              const float dv = xf[a][e] - qf[e];
              sacc += dv * dv;
            } else {
              sacc += xf[a][e] * qf[e];
            }
          }
          acc[a][q] += sacc;
        }
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      float mine = 0.0f;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const float s = wave_sum(acc[a][q]);
        if (q == lane) mine = s;
      }
      const int row = r + a;
      if (lane < NQ && row < ntotal) {
        const float key = (MODE == MODE_L2D) ? mine : -mine;
        if (!FLOOR || lex_less(fk, fi, key, row)) list_insert<KP, int>(lk, li, key, row);
      }
    }
  }

  // In-block merge: the 4 waves' lists of each query meet in LDS (after the
  // queries), wave 0 folds them, and the block writes one list per query.
  float* mk = sq + (int64_t)NQ * ld;      // [4][NQ][KP]
  int* mi = (int*)(mk + 4 * NQ * KP);     // [4][NQ][KP]
  if (lane < NQ) {
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      mk[(w * NQ + lane) * KP + j] = lk[j];
      mi[(w * NQ + lane) * KP + j] = li[j];
    }
  }
  __syncthreads();
  if (w == 0 && lane < NQ) {
#pragma unroll
    for (int o = 1; o < 4; ++o) {
      merge2_sorted<KP, int>(mk + lane * KP, mi + lane * KP, mk + (o * NQ + lane) * KP,
                             mi + (o * NQ + lane) * KP, lk, li);
      if (o < 3) {
#pragma unroll
        for (int j = 0; j < KP; ++j) {
          mk[lane * KP + j] = lk[j];
          mi[lane * KP + j] = li[j];
        }
      }
    }
    float* ok = pkey + ((int64_t)lane * gridDim.x + blockIdx.x) * KP;
    int* oi = pid + ((int64_t)lane * gridDim.x + blockIdx.x) * KP;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      ok[j] = lk[j];
      oi[j] = li[j];
    }
  }
}

template <int NQ, int KP, typename T>
static hipError_t gemv_dispatch_t(int mode, const T* X, const float* Q, int64_t ld,
                                  int ntotal, int nblocks, Partials part, hipStream_t st,
                                  const float* fkey, const int* fid, const int* run) {
  const int ntot16 = (ntotal + 15) & ~15;
  int rpb = (ntot16 + nblocks - 1) / nblocks;
  rpb = (rpb + 15) & ~15;
  const size_t lds = (size_t)NQ * ld * sizeof(float) + (size_t)4 * NQ * KP * 8;
  if (fkey) {
    if constexpr (KP == 64) {
      if (mode == MODE_IP)
        hipLaunchKernelGGL((gemv_topk<NQ, KP, MODE_IP, T, true>), dim3(nblocks), dim3(256), lds,
                           st, X, Q, ld, ntotal, rpb, part.key, part.id, fkey, fid, run);
      else if (mode == MODE_L2D)
        hipLaunchKernelGGL((gemv_topk<NQ, KP, MODE_L2D, T, true>), dim3(nblocks), dim3(256), lds,
                           st, X, Q, ld, ntotal, rpb, part.key, part.id, fkey, fid, run);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  if (mode == MODE_L2D)
    hipLaunchKernelGGL((gemv_topk<NQ, KP, MODE_L2D, T>), dim3(nblocks), dim3(256), lds, st, X, Q,
                       ld, ntotal, rpb, part.key, part.id, nullptr, nullptr, run);
  else if (mode == MODE_IP)
    hipLaunchKernelGGL((gemv_topk<NQ, KP, MODE_IP, T>), dim3(nblocks), dim3(256), lds, st, X, Q,
                       ld, ntotal, rpb, part.key, part.id, nullptr, nullptr, run);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int NQ, int KP>
static hipError_t gemv_dispatch_q(int mode, const void* X, int esize, const float* Q, int64_t ld,
                                  int ntotal, int nblocks, Partials part, hipStream_t st,
                                  const float* fkey, const int* fid, const int* run) {
  if (esize == 4)
    return gemv_dispatch_t<NQ, KP, float>(mode, (const float*)X, Q, ld, ntotal, nblocks, part, st,
                                          fkey, fid, run);
  return gemv_dispatch_t<NQ, KP, uint16_t>(mode, (const uint16_t*)X, Q, ld, ntotal, nblocks, part,
                                           st, fkey, fid, run);
}

template <int KP>
static hipError_t gemv_dispatch(int mode, int nq, const void* X, int esize, const float* Q,
                                int64_t ld, int ntotal, int nblocks, Partials part,
                                hipStream_t st, const float* fkey, const int* fid,
                                const int* run) {
  switch (nq) {
    case 1:
      return gemv_dispatch_q<1, KP>(mode, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    case 2:
      return gemv_dispatch_q<2, KP>(mode, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    case 3:
    case 4:
      return gemv_dispatch_q<4, KP>(mode, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    default:
      return gemv_dispatch_q<8, KP>(mode, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
  }
}

hipError_t launch_gemv_topk(int KP, int mode, int nq, const void* X, int esize, const float* Q,
                            int64_t ld, int ntotal, int nblocks, Partials part, hipStream_t st,
                            const float* fkey, const int* fid, const int* run) {
  if (nq < 1 || nq > kGemvMaxQ || part.KP != KP || part.P != nblocks || (ld * esize) % 16 != 0 ||
      (esize != 4 && esize != 2) || ((fkey == nullptr) != (fid == nullptr)) ||
      (fkey && (KP != 64 || (mode != MODE_IP && mode != MODE_L2D))))
    return hipErrorInvalidValue;
  switch (KP) {
    case 8:
      return gemv_dispatch<8>(mode, nq, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    case 16:
      return gemv_dispatch<16>(mode, nq, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    case 32:
      return gemv_dispatch<32>(mode, nq, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    case 64:
      return gemv_dispatch<64>(mode, nq, X, esize, Q, ld, ntotal, nblocks, part, st, fkey, fid, run);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vs
