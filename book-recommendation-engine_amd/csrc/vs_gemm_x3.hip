// vs_gemm_x3.hip — fp32-accurate fused distance + top-k on the bf16 matrix cores.
//
// Every fp32 value v is split EXACTLY into three bf16 planes
//     hi = bf16(v), mid = bf16(v - hi), lo = v - hi - mid   (hi + mid + lo == v)
// (v has a 24-bit significand; each plane carries 8 of its bits, so the two
// subtractions are exact and lo is representable).  The dot product is then
//     sum_k  x_hi q_hi + x_hi q_mid + x_mid q_hi + x_hi q_lo + x_lo q_hi + x_mid q_mid
// accumulated in fp32 by v_mfma_f32_32x32x16_bf16; each bf16 x bf16 product is
// exact in fp32, and the three dropped terms (mid*lo, lo*mid, lo*lo) are below
// 2^-24 of |x_k q_k| — the size of the rounding error of one fp32 product.  The
// result is therefore an fp32-accurate dot product at 6/16 of the fp32 MFMA
// cost (the bf16 MFMA rate is 16x the fp32 one).  Scores are checked against the
// fp64 oracle with the same tolerance as the plain fp32 kernel.
//
// Database rows: the index keeps the three planes of every row next to the fp32
// rows (built lazily, vs_api.hip), staged with global_load_lds.  Queries: each
// block loads its fp32 query tile slice per stage into registers, splits it,
// and writes the three planes to LDS (the query tile is the smaller operand, so
// the split costs a few VALU ops per MFMA).
//
// Tile: 256 database rows x 128 queries per workgroup of 8 waves (2 per SIMD,
// one workgroup per CU).  Wave w owns rows [128*(w>>2), +128) x queries
// [32*(w&3), +32): four 32x32 accumulators, exactly the per-lane layout of
// gemm_topk (a lane sees one query; register top-k list per lane).
//
// Both operands arrive pre-split (database planes kept by the index, query planes
// built per search) and are staged with global_load_lds_dwordx4 only.  K advances
// 16 elements per stage (one 32x32x16 step, 32-B plane rows); 4 LDS buffers of
// 36 KB keep three stages in flight: stage s+3 is issued right after the barrier
// of stage s, each wave retires its own loads with a COUNTED s_waitcnt vmcnt (never
// 0 inside the K loop), and a raw s_barrier (no __syncthreads, whose fence would
// drain the LDS-DMA queue) publishes the stage.  The 256-row tile halves the query
// re-reads per FLOP relative to a 128-row tile.
#include "vs_device.h"

// Diagnostic builds only (tools/x3_probe.sh): 1 = no MFMA, 2 = no staging loads.
#ifndef VS_X3_PROBE
#define VS_X3_PROBE 0
#endif

namespace vs {

namespace {

constexpr int kXN = 256;     // database rows per tile
constexpr int kXQ = 128;     // queries per tile
constexpr int kXBK = 16;     // elements per stage
constexpr int kRowB = 32;    // bytes per plane row per stage
constexpr int kXPlaneB = kXN * kRowB;               // 8 KB
constexpr int kQPlaneB = kXQ * kRowB;               // 4 KB
constexpr int kBufB = 3 * kXPlaneB + 3 * kQPlaneB;  // 36 KB
constexpr int kNBuf = 4;

// 32-B LDS rows hold 2 chunks of 16 B; chunk c of row r is stored at
// c ^ ((r >> 3) & 1), which spreads each 16-lane ds_read_b128 group of the
// 32-row fragment reads over 16 distinct 16-B slots.
__device__ __forceinline__ int swz32(int r, int c) { return c ^ ((r >> 3) & 1); }

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return (uint32_t)f32_to_bf16_rne(a) | ((uint32_t)f32_to_bf16_rne(b) << 16);
}

__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// Splits 8 floats into three planes of 8 bf16 (16 B each).
__device__ __forceinline__ void split3(const float (&v)[8], uint4& hi, uint4& mid, uint4& lo) {
  uint32_t h[4], m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float a = v[2 * i], b = v[2 * i + 1];
    h[i] = pack_bf16x2(a, b);
    const float ra = a - bf16_lo(h[i]), rb = b - bf16_hi(h[i]);
    m[i] = pack_bf16x2(ra, rb);
    const float sa = ra - bf16_lo(m[i]), sb = rb - bf16_hi(m[i]);
    l[i] = pack_bf16x2(sa, sb);
  }
  hi = make_uint4(h[0], h[1], h[2], h[3]);
  mid = make_uint4(m[0], m[1], m[2], m[3]);
  lo = make_uint4(l[0], l[1], l[2], l[3]);
}

// LDS-DMA of 16 B per lane into the wave-uniform LDS byte address `lds`, issued
// from inline asm so that hipcc does not track it: its own bookkeeping would
// otherwise wait vmcnt(0) before every ds_read of the staging array and drain
// the pipeline.  Completion is counted by hand (wait_vm) and published by the
// raw barrier.  M0 is written and restored inside the statement.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace

template <int KP, int MODE>
__global__ __launch_bounds__(512, 1) void gemm_topk_x3(
    const uint16_t* __restrict__ XP, int64_t pstride, const float* __restrict__ xaux,
    const uint16_t* __restrict__ QP, int64_t qstride, const float* __restrict__ qaux, int64_t ld,
    int nstage, int ntotal, int ntiles, int nsplit, int nqt, int64_t self0,
    float* __restrict__ pkey, int* __restrict__ pid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // kNBuf x kBufB

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2;  // database half of the tile
  const int wq = w & 3;   // query quarter of the tile
  const int h = lane >> 5;
  const int c32 = lane & 31;

  // Bijective XCD remap, as in gemm_topk: logical neighbours share a database split.
  const int nblk = gridDim.x;
  const int b = blockIdx.x;
  int lb;
  {
    const int xcd = b & 7, slot = b >> 3, qq = nblk >> 3, rr = nblk & 7;
    lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  }
  const int qt = lb % nqt;
  const int sp = lb / nqt;
  const int t0 = (int)((int64_t)sp * ntiles / nsplit);
  const int t1 = (int)((int64_t)(sp + 1) * ntiles / nsplit);

  const int qloc = 32 * wq + c32;
  const int gq = qt * kXQ + qloc;
  float qa = 0.0f;
  if constexpr (MODE == MODE_L2 || MODE == MODE_COS) qa = qaux[gq];
  const int selfrow = self0 >= 0 ? (int)(self0 + gq) : -1;

  float lk[KP];
  int li[KP];
  list_init<KP, int>(lk, li);

  // glds geometry: a wave instruction moves 32 rows x 32 B of one plane.
  // X: 3 planes x 8 row groups -> wave w moves group w of each plane (3 per stage).
  // Q: 3 planes x 4 row groups -> waves 0..3 move group w of each plane (3 more).
  const uint32_t prow = (uint32_t)ld * 2u;  // plane row stride in bytes
  const int srow = lane >> 1;
  const uint32_t loff = (uint32_t)srow * prow + (uint32_t)swz32(srow, lane & 1) * 16u;
  const char* qbase = (const char*)(QP + (int64_t)qt * kXQ * ld);
  const bool qstager = w < 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(smem);

  const int fsw = (c32 >> 3) & 1;  // fragment rows 32*s + c32 share (row >> 3) & 1

  for (int t = t0; t < t1; ++t) {
    const char* xbase = (const char*)(XP + (int64_t)t * kXN * ld);
    f32x16 acc[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[s][r] = 0.0f;

    auto issue = [&](int st) {
      if (VS_X3_PROBE == 2) return;
      const uint32_t base = lds0 + (uint32_t)((st & (kNBuf - 1)) * kBufB);
#pragma unroll
      for (int p = 0; p < 3; ++p)
        glds16(xbase + (int64_t)p * pstride * 2 + st * kRowB + (uint32_t)(w * 32) * prow + loff,
               __builtin_amdgcn_readfirstlane(base + p * kXPlaneB + w * 32 * kRowB));
      if (qstager) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          glds16(qbase + (int64_t)p * qstride * 2 + st * kRowB + (uint32_t)(w * 32) * prow + loff,
                 __builtin_amdgcn_readfirstlane(base + 3 * kXPlaneB + p * kQPlaneB +
                                                w * 32 * kRowB));
      }
    };

    // prologue: stages 0..2 in flight
    const int pre = nstage < 3 ? nstage : 3;
    for (int st = 0; st < pre; ++st) issue(st);

    for (int st = 0; st < nstage; ++st) {
      // retire this wave's loads of stage st: later stages issued so far may stay out
      const int ahead = min(2, nstage - 1 - st);
      if (qstager) {
        if (ahead >= 2) wait_vm<12>();
        else if (ahead == 1) wait_vm<6>();
        else wait_vm<0>();
      } else {
        if (ahead >= 2) wait_vm<6>();
        else if (ahead == 1) wait_vm<3>();
        else wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      // every wave has finished reading the buffer of stage st-1: refill it
      if (st + 3 < nstage) issue(st + 3);

      const char* cb = smem + (st & (kNBuf - 1)) * kBufB;
      const int coff = (h ^ fsw) * 16;
      uint4 qf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        qf[p] = *(const uint4*)(cb + 3 * kXPlaneB + p * kQPlaneB + qloc * kRowB + coff);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int xr = 128 * wr + 32 * s + c32;
        uint4 xf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) xf[p] = *(const uint4*)(cb + p * kXPlaneB + xr * kRowB + coff);
        if (VS_X3_PROBE == 1) {
          acc[s][0] += __uint_as_float(xf[0].x ^ xf[1].y ^ xf[2].z ^ qf[0].x ^ qf[1].y ^ qf[2].z);
          continue;
        }
        // the six products above 2^-24: small terms first
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[1]),
                                                        __builtin_bit_cast(bf16x8, qf[1]),
                                                        acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[2]),
                                                        __builtin_bit_cast(bf16x8, qf[0]),
                                                        acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[2]),
                                                        acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[1]),
                                                        __builtin_bit_cast(bf16x8, qf[0]),
                                                        acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[1]),
                                                        acc[s], 0, 0, 0);
        acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[0]),
                                                        acc[s], 0, 0, 0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // all fragment reads done: the LDS is free

    // Epilogue, as in gemm_topk (one 32-row subtile at a time).
    const int r0 = t * kXN + 128 * wr;
    float* spark = (float*)smem;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float tk = lk[KP - 1];
      const int ti = li[KP - 1];
      uint32_t m = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int rb = r0 + 32 * s + 8 * j + 4 * h;
        f32x4 xa = {0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == MODE_L2 || MODE == MODE_COS) xa = *(const f32x4*)(xaux + rb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rb + i;
          const float v = acc[s][j * 4 + i];
          float key;
          if constexpr (MODE == MODE_IP) {
            key = -v;
          } else if constexpr (MODE == MODE_L2) {
            key = l2_from_ip(qa, xa[i], v);
          } else {
            key = -(v * (qa * xa[i]));
          }
          acc[s][j * 4 + i] = key;
          const bool cand = row < ntotal && row != selfrow && lex_less(key, row, tk, ti);
          m |= (uint32_t)cand << (j * 4 + i);
        }
      }
      if (m) {
#pragma unroll
        for (int r = 0; r < 16; ++r) spark[r * 512 + tid] = acc[s][r];
        do {
          const int bi = __builtin_ctz(m);
          m &= m - 1;
          const int row = r0 + 32 * s + (bi & 3) + 8 * (bi >> 2) + 4 * h;
          list_insert<KP, int>(lk, li, spark[bi * 512 + tid], row);
        } while (m);
      }
    }
    __syncthreads();  // the next tile's prologue overwrites the parking area
  }

  const int P = nsplit * 4;
  const int pl = sp * 4 + wr * 2 + h;
  float* ok = pkey + ((int64_t)gq * P + pl) * KP;
  int* oi = pid + ((int64_t)gq * P + pl) * KP;
#pragma unroll
  for (int j = 0; j < KP; ++j) {
    ok[j] = lk[j];
    oi[j] = li[j];
  }
}

template <int KP, int MODE>
static hipError_t x3_launch(const uint16_t* XP, int64_t pstride, const float* xaux,
                            const uint16_t* QP, int64_t qstride, const float* qaux, int64_t ld,
                            int ntotal, int nq_pad, int nsplit, int64_t self0, Partials part,
                            hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_topk_x3<KP, MODE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kNBuf * kBufB);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntiles = (ntotal + kXN - 1) / kXN;
  const int nqt = nq_pad / kXQ;
  hipLaunchKernelGGL((gemm_topk_x3<KP, MODE>), dim3(nqt * nsplit), dim3(512), kNBuf * kBufB, st,
                     XP, pstride, xaux, QP, qstride, qaux, ld, (int)(ld / kXBK), ntotal, ntiles, nsplit, nqt,
                     self0, part.key, part.id);
  return hipGetLastError();
}

template <int KP>
static hipError_t x3_dispatch(int mode, const uint16_t* XP, int64_t pstride, const float* xaux,
                              const uint16_t* QP, int64_t qstride, const float* qaux,
                              int64_t ld, int ntotal, int nq_pad, int nsplit, int64_t self0,
                              Partials part, hipStream_t st) {
  switch (mode) {
    case MODE_IP:
      return x3_launch<KP, MODE_IP>(XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit, self0,
                                    part, st);
    case MODE_L2:
      return x3_launch<KP, MODE_L2>(XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit, self0,
                                    part, st);
    case MODE_COS:
      return x3_launch<KP, MODE_COS>(XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit,
                                     self0, part, st);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_topk_x3(int KP, int mode, const uint16_t* XP, int64_t pstride,
                               const float* xaux, const uint16_t* QP, int64_t qstride,
                               const float* qaux, int64_t ld, int ntotal, int nq_pad, int nsplit,
                               int64_t self0, Partials part, hipStream_t st) {
  if (nq_pad % kXQ != 0 || ld % kXBK != 0 || part.KP != KP || part.P != 4 * nsplit ||
      qstride < (int64_t)nq_pad * ld)
    return hipErrorInvalidValue;
  switch (KP) {
    case 8:
      return x3_dispatch<8>(mode, XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit, self0,
                            part, st);
    case 16:
      return x3_dispatch<16>(mode, XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit, self0,
                             part, st);
    case 32:
      return x3_dispatch<32>(mode, XP, pstride, xaux, QP, qstride, qaux, ld, ntotal, nq_pad, nsplit, self0,
                             part, st);
    default:
      return hipErrorInvalidValue;
  }
}

// Builds the three bf16 planes of rows [r0, r0+n) from the fp32 rows.
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X,
                                                           int64_t ld, int64_t r0, int64_t n,
                                                           uint16_t* __restrict__ XP,
                                                           int64_t pstride) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;  // element index
  const int64_t total = n * ld;
  if (i >= total) return;
  const int64_t e = r0 * ld + i;
  const f32x4 a = *(const f32x4*)(X + e);
  const f32x4 c = *(const f32x4*)(X + e + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  uint4 hi, mid, lo;
  split3(v, hi, mid, lo);
  *(uint4*)(XP + e) = hi;
  *(uint4*)(XP + pstride + e) = mid;
  *(uint4*)(XP + 2 * pstride + e) = lo;
}

hipError_t launch_split_planes(const float* X, int64_t ld, int64_t r0, int64_t n, uint16_t* XP,
                               int64_t pstride, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % 8 != 0) return hipErrorInvalidValue;
  const int64_t nthr = (n * ld + 7) / 8;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, st,
                     X, ld, r0, n, XP, pstride);
  return hipGetLastError();
}

}  // namespace vs
