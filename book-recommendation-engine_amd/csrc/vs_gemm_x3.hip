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
// result is an fp32-accurate dot product at 6/16 of the fp32 MFMA cost (the bf16
// MFMA rate is 16x the fp32 one).  Scores are checked against the fp64 oracle
// with the same tolerance as the plain fp32 kernel.
//
// The split happens INSIDE the kernel, from fp32 data: pre-split planes are 6 B
// per element against 4 B of fp32, and the staging instructions, not the matrix
// cores, bound the first version of this engine, which streamed planes through
// LDS-DMA (profiles/r01_x3_probes.txt: no staging loads 359 ms, all of them
// 536 ms, every load an L2 hit 511 ms).
//
// Tile: 256 database rows x 256 queries per workgroup of 8 waves (two per SIMD,
// one workgroup per CU).  Wave w owns queries [32w, 32w+32) against all 256 rows:
// 8 accumulators of 32x32 (128 registers), and lane l keeps the register top-k
// list of query column l & 31 (lanes l and l+32 see the same query, disjoint rows).
// K advances 16 elements per stage:
//   * database: wave w loads the fp32 slice of rows [32w, 32w+32) (2 x 16 B per
//     lane, one contiguous KiB per instruction in the blocked layout below),
//     splits it and writes the three planes to the stage's LDS image, which all
//     8 waves read as MFMA A fragments (ds_read_b128, conflict-free swizzle);
//   * queries: every wave loads and splits its own 32 queries in registers (the
//     MFMA B fragments) — query data never goes through LDS.
// The data of stage s is fetched one stage early: database slices are loaded at
// the top of stage s-2, split and written to LDS image s%2 at the top of stage
// s-1 and read in stage s; query slices are loaded at the end of stage s-2 and
// split at the end of stage s-1.  Every load is compiler-visible, so its waitcnt
// counts are exact; two LDS images and one barrier per stage.
//
// Blocked fp32 layout (index rows kept by the index, query rows per search; both
// built by block_rows_kernel): element (r, k) of 256-row tile t, K-block b = k/16,
// kk = k%16 sits at
//     (t*nkb + b)*4096 + (((i*8 + (r%256)/32)*2 + h)*32 + r%32)*4 + e,
//     i = kk/8, h = (kk/4)%2, e = kk%4,
// so lane (h*32 + c) of wave w reads row 32w + c with instruction i as one 16-B
// piece of a contiguous KiB, and holds k = 8i + 4h + e in MFMA slot 4i + e — the
// same K permutation on both operands, so the dot product is unchanged.
#include <algorithm>
#include <cstdlib>

#include "vs_device.h"

// Diagnostic builds only (tools/x3_probe.sh; timing only, results are wrong):
// 2 = no global loads in the K loop, 9 = three of the six products.
#ifndef VS_X3_PROBE
#define VS_X3_PROBE 0
#endif

namespace vs {

namespace {

constexpr int kT = 256;                   // database rows (and queries) per tile
constexpr int kKB = 16;                   // K elements per stage
constexpr int kChunkF = kT * kKB;         // floats per (tile, K-block) chunk: 4096
constexpr int kPlaneB = kT * 32;          // one bf16 plane of one stage: 8 KB
constexpr int kStageB = 3 * kPlaneB;      // 24 KB
constexpr int kNBuf = 2;
constexpr int kSparkB = 8 * 16 * 64 * 4;  // epilogue parking, 4 KB per wave
constexpr int kLdsB = kNBuf * kStageB + kSparkB;
constexpr int kX3ChunkTiles = 16;         // database tiles per workgroup per launch

// 32-B LDS rows hold 2 chunks of 16 B; chunk c of row r is stored at
// c ^ ((r >> 3) & 1), which spreads each 16-lane ds_read_b128 group of the
// 32-row fragment reads over 16 distinct 16-B slots.
__device__ __forceinline__ int swz32(int r, int c) { return c ^ ((r >> 3) & 1); }

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk(float a, float b) {  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// Splits 8 floats (two 16-B pieces) into three planes of 8 bf16 (16 B each).
__device__ __forceinline__ void split3(const f32x4& a, const f32x4& b, uint4& hi, uint4& mid,
                                       uint4& lo) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t hh[4], mm[4], ll[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = v[2 * i], x1 = v[2 * i + 1];
    hh[i] = cvt_pk(x0, x1);
    const float r0 = x0 - bf16_lo(hh[i]), r1 = x1 - bf16_hi(hh[i]);
    mm[i] = cvt_pk(r0, r1);
    const float s0 = r0 - bf16_lo(mm[i]), s1 = r1 - bf16_hi(mm[i]);
    ll[i] = cvt_pk(s0, s1);
  }
  hi = make_uint4(hh[0], hh[1], hh[2], hh[3]);
  mid = make_uint4(mm[0], mm[1], mm[2], mm[3]);
  lo = make_uint4(ll[0], ll[1], ll[2], ll[3]);
}

// Publishes this wave's LDS writes and waits for every wave: raw s_barrier (no
// fence, so the global loads in flight are not drained).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ bf16x8 as_bf(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

}  // namespace

template <int KR, int MODE>
__global__ __launch_bounds__(512, 1) void gemm_topk_x3(
    const float* __restrict__ XB, const float* __restrict__ xaux, const uint4* __restrict__ QP,
    const float* __restrict__ qaux, int nqa, int nkb, int ntotal, int ntiles, int nsplit, int nqt,
    int64_t self0, int chunk, int nchunk, int KP, float* __restrict__ pkey,
    int* __restrict__ pid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // kLdsB

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int c32 = lane & 31;

  // Bijective XCD remap: the workgroups of one database split run on one XCD,
  // so each database tile is fetched into that XCD's L2 once for all query tiles.
  const int nblk = gridDim.x;
  const int b = blockIdx.x;
  int lb;
  {
    const int xcd = b & 7, slot = b >> 3, qq = nblk >> 3, rr = nblk & 7;
    lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
  }
  const int qt = lb % nqt;
  const int sp = lb / nqt;
  // this launch's share of the split: chunk `chunk` of `nchunk` (the search is
  // cut into short launches so that the workgroups sharing a split, and thus the
  // database tiles in the XCD's L2, never drift far apart)
  const int s0 = (int)((int64_t)sp * ntiles / nsplit);
  const int s1 = (int)((int64_t)(sp + 1) * ntiles / nsplit);
  const int t0 = s0 + (int)((int64_t)(s1 - s0) * chunk / nchunk);
  const int t1 = s0 + (int)((int64_t)(s1 - s0) * (chunk + 1) / nchunk);

  const int gq = qt * kT + 32 * w + c32;
  float qa = 0.0f;
  if constexpr (MODE == MODE_L2 || MODE == MODE_COS) qa = gq < nqa ? qaux[gq] : 0.0f;
  const int selfrow = self0 >= 0 ? (int)(self0 + gq) : -1;

  const int P = nsplit * 2;
  const int pl = sp * 2 + h;
  float* ok = pkey + ((int64_t)gq * P + pl) * KP;
  int* oi = pid + ((int64_t)gq * P + pl) * KP;
  float lk[KR];
  int li[KR];
  if (chunk == 0) {
    list_init<KR, int>(lk, li);
  } else {  // resume the list the previous chunk wrote
#pragma unroll
    for (int e = 0; e < KR; ++e) {
      lk[e] = ok[e];
      li[e] = oi[e];
    }
  }

  if (t1 > t0) {  // uniform over the workgroup
    // database: per-lane 16-B piece inside a (tile, K-block) chunk (instruction i
    // adds 2048 floats); LDS: this lane's piece (row 32w + c32, half h) and its
    // fragment row c32
    const float* xsrc = XB + (int64_t)(w * 64 + lane) * 4;
    const int wrow = 32 * w + c32;
    const int woff = wrow * 32 + swz32(wrow, h) * 16;
    const int roff = c32 * 32 + swz32(c32, h) * 16;
    // queries: plane p of K-block kb at qsrc[(p * nqt * nkb + kb) * 512]
    const uint4* qsrc = QP + ((int64_t)qt * nkb * 8 + w) * 64 + lane;
    const int64_t qpl = (int64_t)nqt * nkb * 512;

    // database load cursor (tile, K-block) two stages ahead of the compute; past
    // the end it re-reads the last tile (loads stay unconditional)
    int lt = t0, lst = 0;
    auto load_x = [&](f32x4& r0, f32x4& r1) {
      const float* p = xsrc + ((int64_t)min(lt, t1 - 1) * nkb + lst) * kChunkF;
      r0 = *(const f32x4*)p;
      r1 = *(const f32x4*)(p + 2048);
      if (++lst == nkb) {
        lst = 0;
        ++lt;
      }
    };
    auto load_q = [&](int kb, uint4& q0, uint4& q1, uint4& q2) {
      const uint4* p = qsrc + (int64_t)kb * 512;
      q0 = p[0];
      q1 = p[qpl];
      q2 = p[2 * qpl];
    };
    auto write_x = [&](int buf, const f32x4& r0, const f32x4& r1) {
      uint4 p0, p1, p2;
      split3(r0, r1, p0, p1, p2);
      char* base = smem + buf * kStageB + woff;
      *(uint4*)(base) = p0;
      *(uint4*)(base + kPlaneB) = p1;
      *(uint4*)(base + 2 * kPlaneB) = p2;
    };

    // One stage: MFMAs over the image of `buf` with query planes qc*, while
    // stage+1's query planes load into qn*, stage+2's database slice into xn*,
    // and stage+1's database slice (xc*) is split into the other image.
    auto stage = [&](f32x16 (&acc)[8], int buf, int kb_next, const uint4& qc0, const uint4& qc1,
                     const uint4& qc2, uint4& qn0, uint4& qn1, uint4& qn2, const f32x4& xc0,
                     const f32x4& xc1, f32x4& xn0, f32x4& xn1) {
      lds_barrier();  // this stage's image is complete; the previous one is free
      if (VS_X3_PROBE != 2) {
        load_q(kb_next, qn0, qn1, qn2);
        load_x(xn0, xn1);
      }
      const char* cb = smem + buf * kStageB + roff;
      uint4 x0 = *(const uint4*)(cb), x1 = *(const uint4*)(cb + kPlaneB),
            x2 = *(const uint4*)(cb + 2 * kPlaneB);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const char* nb = cb + (i + 1) * 32 * 32;
        f32x16 a = acc[i];
        // the six products above 2^-24; each fragment register is refilled with
        // the next row block's fragment right after its last use
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x0), as_bf(qc0), a, 0, 0, 0);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x0), as_bf(qc1), a, 0, 0, 0);
        if (VS_X3_PROBE != 9)
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x0), as_bf(qc2), a, 0, 0, 0);
        if (i < 7) x0 = *(const uint4*)(nb);
        a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x1), as_bf(qc0), a, 0, 0, 0);
        if (VS_X3_PROBE != 9)
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x1), as_bf(qc1), a, 0, 0, 0);
        if (i < 7) x1 = *(const uint4*)(nb + kPlaneB);
        if (VS_X3_PROBE != 9)
          a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x2), as_bf(qc0), a, 0, 0, 0);
        if (i < 7) x2 = *(const uint4*)(nb + 2 * kPlaneB);
        acc[i] = a;
      }
      write_x(buf ^ 1, xc0, xc1);
    };

    uint4 qa0, qa1, qa2, qb0, qb1, qb2;  // query planes, two stages
    f32x4 xa0, xa1, xb0, xb1;            // raw database slices, two stages
    // prologue: stage 0's image and query planes, stage 1's slice in flight
    f32x4 x00, x01;
    load_x(x00, x01);
    load_q(0, qa0, qa1, qa2);
    load_x(xa0, xa1);
    write_x(0, x00, x01);

    float* spark = (float*)(smem + kNBuf * kStageB) + w * 16 * 64;
    for (int t = t0; t < t1; ++t) {
      f32x16 acc[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][r] = 0.0f;

      // two stages per iteration (nkb is even): the query planes and database
      // slices alternate between the a and b registers, so no copies are needed
      for (int st = 0; st < nkb; st += 2) {
        const int k1 = st + 1, k2 = st + 2 == nkb ? 0 : st + 2;
        stage(acc, 0, k1, qa0, qa1, qa2, qb0, qb1, qb2, xa0, xa1, xb0, xb1);
        stage(acc, 1, k2, qb0, qb1, qb2, qa0, qa1, qa2, xb0, xb1, xa0, xa1);
      }

      // Epilogue (one 32-row block at a time): keys, a 16-bit candidate mask
      // against the lane's current worst entry, and insertion of the flagged
      // values only (after the first tiles almost nothing passes).
      const int r0 = t * kT;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        f32x4 xa[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          xa[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (MODE == MODE_L2 || MODE == MODE_COS)
            xa[jj] = *(const f32x4*)(xaux + r0 + 32 * i + 8 * jj + 4 * h);
        }
        const float tk = lk[KR - 1];
        const int ti = li[KR - 1];
        uint32_t m = 0;
        f32x16 v16 = acc[i];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int rb = r0 + 32 * i + 8 * jj + 4 * h;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = rb + e;
            const float v = v16[jj * 4 + e];
            float key;
            if constexpr (MODE == MODE_IP) {
              key = -v;
            } else if constexpr (MODE == MODE_L2) {
              key = l2_from_ip(qa, xa[jj][e], v);
            } else {
              key = -(v * (qa * xa[jj][e]));
            }
            v16[jj * 4 + e] = key;
            const bool cand = row < ntotal && row != selfrow && lex_less(key, row, tk, ti);
            m |= (uint32_t)cand << (jj * 4 + e);
          }
        }
        if (m) {
#pragma unroll
          for (int r = 0; r < 16; ++r) spark[r * 64 + lane] = v16[r];
          do {
            const int bi = __builtin_ctz(m);
            m &= m - 1;
            const int row = r0 + 32 * i + (bi & 3) + 8 * (bi >> 2) + 4 * h;
            list_insert<KR, int>(lk, li, spark[bi * 64 + lane], row);
          } while (m);
        }
      }
    }
  }

#pragma unroll
  for (int e = 0; e < KR; ++e) {
    ok[e] = lk[e];
    oi[e] = li[e];
  }
  for (int e = KR; e < KP; ++e) {  // the merge reads KP entries per list
    ok[e] = FLT_MAX;
    oi[e] = -1;
  }
}

template <int KR, int MODE>
static hipError_t x3_launch(const X3Args& a, Partials part, hipStream_t st, int* ndispatch) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_topk_x3<KR, MODE>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kLdsB);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntiles = (a.ntotal + kT - 1) / kT;
  const int nqt = a.nq_pad / kT;
  // chunks of about kX3ChunkTiles tiles per workgroup (VS_X3_CHUNK_TILES overrides)
  static const int chunk_tiles = [] {
    const char* e = getenv("VS_X3_CHUNK_TILES");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : kX3ChunkTiles;
  }();
  const int per_block = (ntiles + a.nsplit - 1) / a.nsplit;
  const int nchunk = std::max(1, (per_block + chunk_tiles - 1) / chunk_tiles);
  for (int c = 0; c < nchunk; ++c) {
    hipLaunchKernelGGL((gemm_topk_x3<KR, MODE>), dim3(nqt * a.nsplit), dim3(512), kLdsB, st,
                       a.XB, a.xaux, a.QP, a.qaux, a.nqa, (int)(a.ld / kKB), a.ntotal, ntiles,
                       a.nsplit, nqt, a.self0, c, nchunk, part.KP, part.key, part.id);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (ndispatch) *ndispatch = nchunk;
  return hipSuccess;
}

template <int KR>
static hipError_t x3_dispatch(int mode, const X3Args& a, Partials part, hipStream_t st,
                              int* ndispatch) {
  switch (mode) {
    case MODE_IP:
      return x3_launch<KR, MODE_IP>(a, part, st, ndispatch);
    case MODE_L2:
      return x3_launch<KR, MODE_L2>(a, part, st, ndispatch);
    case MODE_COS:
      return x3_launch<KR, MODE_COS>(a, part, st, ndispatch);
    default:
      return hipErrorInvalidValue;
  }
}

// Longer lists do not fit the register file beside the 128 accumulators (KR=32
// spills ~100 registers into the K loop): those searches take the fp32 engine.
int x3_list_len(int need) {
  return need <= 8 ? 8 : need <= 12 ? 12 : need <= 16 ? 16 : need <= 20 ? 20 : need <= 24 ? 24 : 0;
}

hipError_t launch_gemm_topk_x3(int KR, int mode, const X3Args& a, Partials part, hipStream_t st,
                               int* ndispatch) {
  // ld % 32: an even number of K-blocks per tile keeps the LDS image parity of a
  // stage equal to its K-block parity across tiles
  if (a.nq_pad % kT != 0 || a.ld % (2 * kKB) != 0 || KR > part.KP || part.P != 2 * a.nsplit ||
      a.nsplit < 1)
    return hipErrorInvalidValue;
  switch (KR) {
    case 8:
      return x3_dispatch<8>(mode, a, part, st, ndispatch);
    case 12:
      return x3_dispatch<12>(mode, a, part, st, ndispatch);
    case 16:
      return x3_dispatch<16>(mode, a, part, st, ndispatch);
    case 20:
      return x3_dispatch<20>(mode, a, part, st, ndispatch);
    case 24:
      return x3_dispatch<24>(mode, a, part, st, ndispatch);
    default:
      return hipErrorInvalidValue;
  }
}

// Copies fp32 rows [r0, r0+n) (row-major, stride ld) into the blocked layout
// described at the top of this file.  One thread moves one 16-B piece.
__global__ __launch_bounds__(256) void block_rows_kernel(const float* __restrict__ X, int64_t ld,
                                                         int64_t r0, int64_t n,
                                                         float* __restrict__ XB) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;  // piece index
  const int64_t per_row = ld / 4;
  if (p >= n * per_row) return;
  const int64_t r = r0 + p / per_row;
  const int64_t k = (p % per_row) * 4;
  const f32x4 v = *(const f32x4*)(X + r * ld + k);
  const int64_t t = r / kT, rr = r % kT, bk = k / kKB, kk = k % kKB;
  const int64_t i = kk >> 3, hh = (kk >> 2) & 1;
  const int64_t o =
      (t * (ld / kKB) + bk) * kChunkF + (((i * 8 + rr / 32) * 2 + hh) * 32 + rr % 32) * 4;
  *(f32x4*)(XB + o) = v;
}

// Splits fp32 query rows [0, n) (stride ld) into the three bf16 planes of the
// MFMA B fragments: uint4 ((p*nqt + r/256)*nkb + kb)*512 + ((r%256)/32)*64 + lane,
// lane = h*32 + r%32, holding k = 16kb + {4h..4h+3, 8+4h..8+4h+3} (the K
// permutation of the blocked database rows).  One thread per (row, kb, h).
__global__ __launch_bounds__(256) void split_queries_kernel(const float* __restrict__ Q,
                                                            int64_t ld, int64_t n, int nqt,
                                                            uint4* __restrict__ QP) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nkb = ld / kKB;
  if (p >= n * nkb * 2) return;
  const int64_t r = p / (nkb * 2);
  const int64_t kb = (p / 2) % nkb;
  const int hh = (int)(p & 1);
  const float* src = Q + r * ld + kb * kKB + 4 * hh;
  const f32x4 a = *(const f32x4*)src;
  const f32x4 c = *(const f32x4*)(src + 8);
  uint4 p0, p1, p2;
  split3(a, c, p0, p1, p2);
  const int64_t o = ((r / kT) * nkb + kb) * 512 + ((r % kT) / 32) * 64 + hh * 32 + r % 32;
  const int64_t pl = (int64_t)nqt * nkb * 512;
  QP[o] = p0;
  QP[o + pl] = p1;
  QP[o + 2 * pl] = p2;
}

hipError_t launch_split_queries(const float* Q, int64_t ld, int64_t n, int nq_pad, uint4* QP,
                                hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % kKB != 0 || nq_pad % kT != 0 || n > nq_pad) return hipErrorInvalidValue;
  const int64_t items = n * (ld / kKB) * 2;
  hipLaunchKernelGGL(split_queries_kernel, dim3((unsigned)((items + 255) / 256)), dim3(256), 0, st,
                     Q, ld, n, nq_pad / kT, QP);
  return hipGetLastError();
}

hipError_t launch_block_rows(const float* X, int64_t ld, int64_t r0, int64_t n, float* XB,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % kKB != 0) return hipErrorInvalidValue;
  const int64_t pieces = n * (ld / 4);
  hipLaunchKernelGGL(block_rows_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, st,
                     X, ld, r0, n, XB);
  return hipGetLastError();
}

}  // namespace vs
