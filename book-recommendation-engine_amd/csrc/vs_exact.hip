// vs_exact.hip — the exact-key stream: top-k by the rescoring's own keys for
// the queries no proof settles (the staged engine's last resort).
//
// The filter stages prove their candidate sets; the last
// stage (vs_api.hip run_gemm_rescored) takes the fp32 MFMA GEMM's top-KF and
// proves them with the fp32 GEMM's own error bound.  A query whose k-th best
// row has more than KF - k rows inside that bound (dense near-ties: copies of
// a row spaced below the fp32 GEMM's rounding) cannot be proven from any
// fp32 candidate list of KF rows; this kernel ranks EVERY row by the exact key
// the rescoring computes — fp64 sums of the fp32 products (exact products),
// rounded once, then the metric's key formula (vs_gemm_x1.hip exact_key) —
// so its lists are the answer itself, with no bound.  Each lane sums the
// 16-B chunks c = lane, lane + 64, ... of a row with fma in element order and
// the wave reduces by xor-shuffles 32 .. 1: wave_dot's order, so a row's key is
// bit-identical to the one verify_rescore gives it.
//
// With a floor per query (fkey / fid: the paged engine's previous page) it is
// the exact-key form of a page: the staged engine's last stage past 64
// candidates (vs_api.hip run_paged, gathered) pages each query's order of exact
// keys 64 entries at a time.
//
// Layout: one workgroup per block of rows (4 waves, each wave 4 rows at a
// time, lane l reading chunk l of each: 1 KiB per wave instruction, coalesced),
// persistent over the gathered queries in groups of NQ (their rows staged in
// LDS): blocks of a launch with nothing to do exit at once, so the launch costs
// ~nothing when no query reaches it (the host never reads the count).  HBM-bound:
// N·d·4 bytes per group of NQ queries (10M x 1536: ~10 ms per 8 queries).
#include "vs_device.h"

namespace vs {

template <int NQ, int KP, int MODE>
__global__ __launch_bounds__(256) void exact_stream_topk(
    const float* __restrict__ X, const float* __restrict__ xn, int64_t ld, int ntotal,
    int rows_per_block, const float* __restrict__ Q, const float* __restrict__ qaux,
    const int* __restrict__ qrow, const float* __restrict__ xinv, const int* __restrict__ slots,
    const int* __restrict__ count, int s0, int nslot, float* __restrict__ pkey,
    int* __restrict__ pid, const float* __restrict__ fkey, const int* __restrict__ fid) {
  extern __shared__ __attribute__((aligned(16))) float sq[];  // [NQ][ld], then list merge
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int n = min(*count - s0, nslot);  // this launch's slots of the list
  if (n <= 0) return;                      // uniform
  const int cpr = (int)(ld / 4);
  const int rb0 = blockIdx.x * rows_per_block;
  const int rb1 = min(rb0 + rows_per_block, ntotal);
  float* mk = sq + (int64_t)NQ * ld;  // [4][NQ][KP]
  int* mi = (int*)(mk + 4 * NQ * KP);

  for (int g = 0; g * NQ < n; ++g) {
    __syncthreads();  // the previous group's readers of sq / mk are done
    for (int i = tid; i < NQ * cpr; i += 256) {
      const int q = i / cpr, c = i - q * cpr;
      const int j = g * NQ + q;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (j < n) v = *(const f32x4*)(Q + (int64_t)slots[s0 + j] * ld + 4 * c);
      *(f32x4*)(sq + (int64_t)q * ld + 4 * c) = v;
    }
    __syncthreads();
    const int jq = g * NQ + (lane < NQ ? lane : 0);
    const int sl = jq < n ? slots[s0 + jq] : 0;
    float qa = 0.0f;
    int self = -1;
    // a page's floor (the paged engine): only entries lexicographically after
    // the previous page's last one enter; none: (-inf, -1)
    float fk = -INFINITY;
    int fi = -1;
    if (lane < NQ && jq < n) {
      if constexpr (MODE == MODE_L2 || MODE == MODE_COS) qa = qaux[sl];
      if (qrow) self = qrow[sl];
      if (fkey) {
        fk = fkey[sl];
        fi = fid[sl];
      }
    }
    float lk[KP];
    int li[KP];
    list_init<KP, int>(lk, li);
    for (int r = rb0 + 4 * w; r < rb1; r += 16) {
      double acc[4][NQ];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[a][q] = 0.0;
      for (int c = lane; c < cpr; c += 64) {
        f32x4 xv[4];
#pragma unroll
        for (int a = 0; a < 4; ++a)
          xv[a] = r + a < rb1 ? *(const f32x4*)(X + (int64_t)(r + a) * ld + 4 * c)
                              : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const f32x4 qv = *(const f32x4*)(sq + (int64_t)q * ld + 4 * c);
#pragma unroll
          for (int a = 0; a < 4; ++a) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              if constexpr (MODE == MODE_L2D) {
                const double t = (double)xv[a][e] - (double)qv[e];
                acc[a][q] = fma(t, t, acc[a][q]);
              } else {
                acc[a][q] = fma((double)xv[a][e], (double)qv[e], acc[a][q]);
              }
            }
          }
        }
      }
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        double mine = 0.0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          double s = acc[a][q];
          for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
          if (q == lane) mine = s;
        }
        const int row = r + a;
        if (lane < NQ && jq < n && row < rb1 && row != self) {
          const float ip = (float)mine;
          float key;
          if constexpr (MODE == MODE_IP) {
            key = -ip;
          } else if constexpr (MODE == MODE_L2) {
            key = l2_from_ip(qa, xn[row], ip);
          } else if constexpr (MODE == MODE_COS) {
            key = -(ip * (qa * xinv[row]));
          } else {
            key = ip;  // the rounded exact sum of (x - q)^2
          }
          if (lex_less(fk, fi, key, row)) list_insert<KP, int>(lk, li, key, row);
        }
      }
    }
    // the 4 waves' lists of each query meet in LDS; wave 0 folds them
    if (lane < NQ) {
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        mk[(w * NQ + lane) * KP + j] = lk[j];
        mi[(w * NQ + lane) * KP + j] = li[j];
      }
    }
    __syncthreads();
    if (w == 0 && lane < NQ && jq < n) {
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
      float* ok = pkey + ((int64_t)jq * gridDim.x + blockIdx.x) * KP;
      int* oi = pid + ((int64_t)jq * gridDim.x + blockIdx.x) * KP;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        ok[j] = lk[j];
        oi[j] = li[j];
      }
    }
  }
}

template <int NQ, int KP>
static hipError_t exact_dispatch_mode(int mode, const ExactStreamArgs& a, Partials part,
                                      hipStream_t st) {
  const int rpb = (int)((a.ntotal + part.P - 1) / part.P);
  const size_t lds = (size_t)NQ * a.ld * sizeof(float) + (size_t)4 * NQ * KP * 8;
#define VS_EXACT(MD)                                                                            \
  hipLaunchKernelGGL((exact_stream_topk<NQ, KP, MD>), dim3(part.P), dim3(256), lds, st, a.X,     \
                     a.xn, a.ld, a.ntotal, rpb, a.Q, a.qaux, a.qrow, a.xinv, a.slots, a.count,  \
                     a.s0, a.nslot, part.key, part.id, a.fkey, a.fid)
  switch (mode) {
    case MODE_IP:
      VS_EXACT(MODE_IP);
      break;
    case MODE_L2:
      VS_EXACT(MODE_L2);
      break;
    case MODE_L2D:
      VS_EXACT(MODE_L2D);
      break;
    case MODE_COS:
      VS_EXACT(MODE_COS);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef VS_EXACT
  return hipGetLastError();
}

template <int KP>
static hipError_t exact_dispatch(int mode, const ExactStreamArgs& a, Partials part,
                                 hipStream_t st) {
  switch (exact_stream_nq(a.ld)) {
    case 8:
      return exact_dispatch_mode<8, KP>(mode, a, part, st);
    case 4:
      return exact_dispatch_mode<4, KP>(mode, a, part, st);
    case 2:
      return exact_dispatch_mode<2, KP>(mode, a, part, st);
    case 1:
      return exact_dispatch_mode<1, KP>(mode, a, part, st);
    default:
      return hipErrorInvalidValue;
  }
}

int exact_stream_nq(int64_t ld) {
  for (int nq = 8; nq >= 1; nq >>= 1)
    if ((size_t)nq * ld * sizeof(float) + (size_t)4 * nq * 64 * 8 <= 64 * 1024) return nq;
  return 0;
}

hipError_t launch_exact_stream(int KP, int mode, const ExactStreamArgs& a, Partials part,
                               hipStream_t st) {
  if (part.KP != KP || part.P < 1 || a.ld % 4 != 0 || a.ntotal < 1 || a.nslot < 1 ||
      exact_stream_nq(a.ld) == 0 || (mode == MODE_COS && (!a.xinv || !a.qaux)) ||
      (mode == MODE_L2 && (!a.xn || !a.qaux)))
    return hipErrorInvalidValue;
  switch (KP) {
    case 8:
      return exact_dispatch<8>(mode, a, part, st);
    case 16:
      return exact_dispatch<16>(mode, a, part, st);
    case 32:
      return exact_dispatch<32>(mode, a, part, st);
    case 64:
      return exact_dispatch<64>(mode, a, part, st);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vs
