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
// Tile: 256 database rows x 256 queries per workgroup of 4 waves (one per SIMD,
// one workgroup per CU).  Wave w owns all 256 rows x queries [64w, 64w+64): 8 x 2
// accumulators of 32x32 (256 registers: the accumulator file), so a lane sees
// TWO queries (columns lane&31 of its two query blocks) and keeps two register
// top-k lists.  The square tile moves 48 KB of planes per 384 MFMAs, a third less
// per MFMA than a 256x128 tile (the staging path, not the matrix cores, bounded
// the 256x128 version: profiles/r01_x3_probe.txt).
//
// Both operands arrive pre-split in a K-blocked layout (database planes kept by
// the index, query planes built per search; split_planes_kernel) and are staged
// with global_load_lds_dwordx4 only.  K advances 16 elements per stage (one
// 32x32x16 step); 3 LDS buffers of 48 KB keep two stages in flight: stage s+2 is
// issued right after the barrier of stage s, each wave retires its own loads with
// a COUNTED s_waitcnt vmcnt (never 0 inside the K loop), and a raw s_barrier
// publishes the stage.
#include <algorithm>
#include <cstdlib>

#include "vs_device.h"

// Diagnostic builds only (tools/x3_probe.sh; timing only, results are wrong):
// 1 = no MFMA, 2 = no staging loads, 3 = no vmcnt wait, 4 = no stage barrier,
// 5 = neither, 6 = database planes only, 7 = query planes only, 8 = every load
// from tile 0 (L2-resident).
#ifndef VS_X3_PROBE
#define VS_X3_PROBE 0
#endif

namespace vs {

namespace {

constexpr int kXN = 256;     // database rows per tile
constexpr int kXQ = 256;     // queries per tile
constexpr int kXBK = 16;     // elements per stage
constexpr int kRowB = 32;    // bytes per plane row per stage
constexpr int kXPlaneB = kXN * kRowB;               // 8 KB
constexpr int kQPlaneB = kXQ * kRowB;               // 8 KB
constexpr int kBufB = 3 * kXPlaneB + 3 * kQPlaneB;  // 48 KB
constexpr int kNBuf = 3;
constexpr int kX3ChunkTiles = 16;  // database tiles per workgroup per launch
constexpr int kX3Waves = 8;

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
// Same with the non-temporal hint (streamed operand: keep it from evicting
// lines that other workgroups of the XCD are about to re-read).
__device__ __forceinline__ void glds16_nt(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}
#ifndef VS_X3_QNT
#define VS_X3_QNT 0
#endif

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace

template <int KP, int MODE, int NW>
__global__ __launch_bounds__(64 * NW, 1) void gemm_topk_x3(
    const uint16_t* __restrict__ XP, int64_t pstride, const float* __restrict__ xaux,
    const uint16_t* __restrict__ QP, int64_t qstride, const float* __restrict__ qaux, int nqa,
    int nstage, int ntotal, int ntiles, int nsplit, int nqt, int64_t self0, int chunk,
    int nchunk, float* __restrict__ pkey, int* __restrict__ pid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // kNBuf x kBufB

  // NW = 4: wave w owns queries [64w, 64w+64) (two 32-query blocks, two lists
  // per lane, 256 accumulator registers, one wave per SIMD).  NW = 8: wave w owns
  // queries [32w, 32w+32) (one list per lane, 128 accumulator registers, two
  // waves per SIMD).  Every wave covers all 256 rows of the tile.
  constexpr int NJ = 8 / NW;       // 32-query blocks per wave
  constexpr int NPART = 24 / NW;   // staging parts (2 LDS-DMA each) per wave per stage
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
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
  // this launch's share of the split: chunk `chunk` of `nchunk` (the search is
  // cut into short launches so that the workgroups sharing a split, and thus
  // the database tiles in the XCD's L2, never drift far apart)
  const int s0 = (int)((int64_t)sp * ntiles / nsplit);
  const int s1 = (int)((int64_t)(sp + 1) * ntiles / nsplit);
  const int t0 = s0 + (int)((int64_t)(s1 - s0) * chunk / nchunk);
  const int t1 = s0 + (int)((int64_t)(s1 - s0) * (chunk + 1) / nchunk);

  int gq[NJ];
  float qa[NJ];
  int selfrow[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    gq[j] = qt * kXQ + 32 * (NJ * w + j) + c32;
    qa[j] = 0.0f;
    if constexpr (MODE == MODE_L2 || MODE == MODE_COS) qa[j] = gq[j] < nqa ? qaux[gq[j]] : 0.0f;
    selfrow[j] = self0 >= 0 ? (int)(self0 + gq[j]) : -1;
  }

  const int P = nsplit * 2;
  const int pl = sp * 2 + h;
  float lk[NJ][KP];
  int li[NJ][KP];
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    if (chunk == 0) {
      list_init<KP, int>(lk[j], li[j]);
    } else {  // resume the lists the previous chunk wrote
      const float* ok = pkey + ((int64_t)gq[j] * P + pl) * KP;
      const int* oi = pid + ((int64_t)gq[j] * P + pl) * KP;
#pragma unroll
      for (int e = 0; e < KP; ++e) {
        lk[j][e] = ok[e];
        li[j][e] = oi[e];
      }
    }
  }

  // glds geometry: a wave instruction moves 32 rows x 32 B of one plane; each
  // plane's stage slice is 8 row groups, wave w moves groups 2w and 2w+1 of the
  // three database and the three query planes (12 instructions per stage).
  // Planes are K-blocked: a stage's slice of one plane is one contiguous block
  // of 256 rows x 32 B, so every fetched line is used whole.
  const int srow = lane >> 1;
  const uint32_t loff = (uint32_t)srow * kRowB + (uint32_t)swz32(srow, lane & 1) * 16u;
  const char* qbase = (const char*)(QP + (int64_t)(VS_X3_PROBE == 8 ? 0 : qt) * nstage * kXQ * 16);
  const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(smem);
  const int fsw = (c32 >> 3) & 1;  // fragment rows 32*i + c32 share (row >> 3) & 1
  const int coff = (h ^ fsw) * 16;

  // The stage pipeline runs continuously over the block's tiles: the issue
  // cursor (tile it, stage ist, buffer ibuf) stays two stages ahead of the
  // compute cursor, also across tile boundaries, so the epilogue of one tile
  // overlaps the first loads of the next and no tile restarts the pipeline.
  const int nst_total = (t1 - t0) * nstage;
  int it = t0, ist = 0, ibuf = 0;
  // LDS-DMA v (0 .. 2*NPART-1) of the cursor stage: operand v & 1 (database or
  // query planes), plane (v >> 1) / NJ, row group NJ*w + (v >> 1) % NJ.  They are
  // spread evenly over a stage's MFMA groups: bursts of LDS-DMA writes delay the
  // fragment reads the MFMAs wait on.
  auto issue_one = [&](int v) {
    if (VS_X3_PROBE == 2) return;
    if (VS_X3_PROBE == 6 && (v & 1)) return;
    if (VS_X3_PROBE == 7 && !(v & 1)) return;
    const uint32_t base = lds0 + (uint32_t)(ibuf * kBufB);
    const int u = v >> 1;
    const int p = u / NJ;
    const int grp = NJ * w + u % NJ;
    if ((v & 1) == 0) {
      const char* xb = (const char*)(XP + (int64_t)(VS_X3_PROBE == 8 ? 0 : it) * nstage * kXN * 16);
      glds16(xb + (int64_t)p * pstride * 2 + ist * kXPlaneB + grp * 1024 + loff,
             __builtin_amdgcn_readfirstlane(base + p * kXPlaneB + grp * 1024));
    } else {
      const char* qsrc = qbase + (int64_t)p * qstride * 2 + ist * kQPlaneB + grp * 1024 + loff;
      const uint32_t qdst =
          __builtin_amdgcn_readfirstlane(base + 3 * kXPlaneB + p * kQPlaneB + grp * 1024);
      if (VS_X3_QNT) glds16_nt(qsrc, qdst);
      else glds16(qsrc, qdst);
    }
  };
  auto advance = [&]() {
    ibuf = ibuf == kNBuf - 1 ? 0 : ibuf + 1;
    if (++ist == nstage) {
      ist = 0;
      ++it;
    }
  };
  // prologue: two stages in flight
  for (int g = 0; g < 2 && g < nst_total; ++g) {
    for (int v = 0; v < 2 * NPART; ++v) issue_one(v);
    advance();
  }

  int g = 0;     // compute cursor (stage index over the block's tiles)
  int cbuf = 0;  // its buffer
  for (int t = t0; t < t1; ++t) {
    f32x16 acc[8][NJ];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    for (int st = 0; st < nstage; ++st, ++g) {
      // retire this wave's loads of stage g (stage g+1 may stay in flight)
      if (VS_X3_PROBE != 3 && VS_X3_PROBE != 5) {
        if (g + 1 < nst_total) wait_vm<2 * NPART>();
        else wait_vm<0>();
      }
      if (VS_X3_PROBE != 4 && VS_X3_PROBE != 5) __builtin_amdgcn_s_barrier();
      // every wave has finished reading the buffer of stage g-1: it is refilled
      // with stage g+2 during this stage's MFMAs
      const bool refill = g + 2 < nst_total;

      const char* cb = smem + cbuf * kBufB;
      uint4 qf[NJ][3], xf[3], xn[3];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          qf[j][p] = *(const uint4*)(cb + 3 * kXPlaneB + p * kQPlaneB +
                                     (32 * (NJ * w + j) + c32) * kRowB + coff);
#pragma unroll
      for (int p = 0; p < 3; ++p) xf[p] = *(const uint4*)(cb + p * kXPlaneB + c32 * kRowB + coff);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        // next row block's fragments are requested before this block's MFMAs
        if (i < 7) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            xn[p] = *(const uint4*)(cb + p * kXPlaneB + (32 * (i + 1) + c32) * kRowB + coff);
        }
        if (refill) {
#pragma unroll
          for (int v = 0; v < 2 * NPART; ++v)
            if (v * 8 / (2 * NPART) == i) issue_one(v);
        }
        if (VS_X3_PROBE == 1) {
          acc[i][0][0] += __uint_as_float(xf[0].x ^ xf[1].y ^ xf[2].z ^ qf[0][0].x ^
                                          qf[NJ - 1][1].y ^ qf[0][2].z);
        } else {
#pragma unroll
          for (int j = 0; j < NJ; ++j) {
            // the six products above 2^-24: small terms first
            f32x16 a = acc[i][j];
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[1]),
                                                        __builtin_bit_cast(bf16x8, qf[j][1]), a,
                                                        0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[2]),
                                                        __builtin_bit_cast(bf16x8, qf[j][0]), a,
                                                        0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[j][2]), a,
                                                        0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[1]),
                                                        __builtin_bit_cast(bf16x8, qf[j][0]), a,
                                                        0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[j][1]), a,
                                                        0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                        __builtin_bit_cast(bf16x8, qf[j][0]), a,
                                                        0, 0, 0);
            acc[i][j] = a;
          }
        }
        if (i < 7) {
#pragma unroll
          for (int p = 0; p < 3; ++p) xf[p] = xn[p];
        }
      }
      if (refill) advance();
      cbuf = cbuf == kNBuf - 1 ? 0 : cbuf + 1;
    }
    // every wave has finished reading the last stage's buffer, which is not
    // refilled before the next barrier: it parks this tile's epilogue values
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int lbuf = cbuf == 0 ? kNBuf - 1 : cbuf - 1;

    // Epilogue, as in gemm_topk (one 32-row block at a time).
    const int r0 = t * kXN;
    float* spark = (float*)(smem + lbuf * kBufB) + w * 16 * 64;  // 4 KB per wave
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f32x4 xa[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        xa[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == MODE_L2 || MODE == MODE_COS)
          xa[jj] = *(const f32x4*)(xaux + r0 + 32 * i + 8 * jj + 4 * h);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float tk = lk[j][KP - 1];
        const int ti = li[j][KP - 1];
        uint32_t m = 0;
        f32x16 v16 = acc[i][j];
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
              key = l2_from_ip(qa[j], xa[jj][e], v);
            } else {
              key = -(v * (qa[j] * xa[jj][e]));
            }
            v16[jj * 4 + e] = key;
            const bool cand = row < ntotal && row != selfrow[j] && lex_less(key, row, tk, ti);
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
            list_insert<KP, int>(lk[j], li[j], spark[bi * 64 + lane], row);
          } while (m);
        }
      }
    }
  }

#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    float* ok = pkey + ((int64_t)gq[j] * P + pl) * KP;
    int* oi = pid + ((int64_t)gq[j] * P + pl) * KP;
#pragma unroll
    for (int e = 0; e < KP; ++e) {
      ok[e] = lk[j][e];
      oi[e] = li[j][e];
    }
  }
}

template <int KP, int MODE, int NW>
static hipError_t x3_launch_nw(const X3Args& a, Partials part, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)gemm_topk_x3<KP, MODE, NW>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, kNBuf * kBufB);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int ntiles = (a.ntotal + kXN - 1) / kXN;
  const int nqt = a.nq_pad / kXQ;
  // chunks of about kX3ChunkTiles tiles per workgroup (VS_X3_CHUNK_TILES overrides)
  static const int chunk_tiles = [] {
    const char* e = getenv("VS_X3_CHUNK_TILES");
    const int v = e ? atoi(e) : 0;
    return v > 0 ? v : kX3ChunkTiles;
  }();
  const int per_block = (ntiles + a.nsplit - 1) / a.nsplit;
  const int nchunk = std::max(1, (per_block + chunk_tiles - 1) / chunk_tiles);
  for (int c = 0; c < nchunk; ++c) {
    hipLaunchKernelGGL((gemm_topk_x3<KP, MODE, NW>), dim3(nqt * a.nsplit), dim3(64 * NW),
                       kNBuf * kBufB, st, a.XP, a.pstride, a.xaux, a.QP, a.qstride, a.qaux, a.nqa,
                       (int)(a.ld / kXBK), a.ntotal, ntiles, a.nsplit, nqt, a.self0, c, nchunk,
                       part.key, part.id);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// VS_X3_WAVES=4|8 selects the wave layout (A/B runs); default kX3Waves.
template <int KP, int MODE>
static hipError_t x3_launch(const X3Args& a, Partials part, hipStream_t st) {
  static const int nw = [] {
    const char* e = getenv("VS_X3_WAVES");
    return e && atoi(e) == 4 ? 4 : e && atoi(e) == 8 ? 8 : kX3Waves;
  }();
  return nw == 4 ? x3_launch_nw<KP, MODE, 4>(a, part, st) : x3_launch_nw<KP, MODE, 8>(a, part, st);
}

template <int KP>
static hipError_t x3_dispatch(int mode, const X3Args& a, Partials part, hipStream_t st) {
  switch (mode) {
    case MODE_IP:
      return x3_launch<KP, MODE_IP>(a, part, st);
    case MODE_L2:
      return x3_launch<KP, MODE_L2>(a, part, st);
    case MODE_COS:
      return x3_launch<KP, MODE_COS>(a, part, st);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_topk_x3(int KP, int mode, const X3Args& a, Partials part, hipStream_t st) {
  if (a.nq_pad % kXQ != 0 || a.ld % kXBK != 0 || part.KP != KP || part.P != 2 * a.nsplit ||
      a.qstride < (int64_t)a.nq_pad * a.ld || a.nsplit < 1)
    return hipErrorInvalidValue;
  switch (KP) {
    case 8:
      return x3_dispatch<8>(mode, a, part, st);
    case 16:
      return x3_dispatch<16>(mode, a, part, st);
    case 32:
      return x3_dispatch<32>(mode, a, part, st);
    default:
      return hipErrorInvalidValue;
  }
}

// Builds the three bf16 planes of rows [r0, r0+n) from the fp32 rows, in the
// K-blocked layout the GEMM stages from: element (r, k) of a plane sits at
//   ((r / T * (ld / 16) + k / 16) * T + r % T) * 16 + k % 16
// with T = tile_rows (= kXN = kXQ = 256 for index and query planes).
__global__ __launch_bounds__(256) void split_planes_kernel(const float* __restrict__ X,
                                                           int64_t ld, int64_t r0, int64_t n,
                                                           uint16_t* __restrict__ XP,
                                                           int64_t pstride, int tile_rows) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;  // element index
  const int64_t total = n * ld;
  if (i >= total) return;
  const int64_t r = r0 + i / ld;
  const int64_t k = i % ld;
  const float* src = X + r * ld + k;
  const f32x4 a = *(const f32x4*)(src);
  const f32x4 c = *(const f32x4*)(src + 4);
  const float v[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  uint4 hi, mid, lo;
  split3(v, hi, mid, lo);
  const int64_t o =
      ((r / tile_rows * (ld / 16) + k / 16) * tile_rows + r % tile_rows) * 16 + (k % 16);
  *(uint4*)(XP + o) = hi;
  *(uint4*)(XP + pstride + o) = mid;
  *(uint4*)(XP + 2 * pstride + o) = lo;
}

hipError_t launch_split_planes(const float* X, int64_t ld, int64_t r0, int64_t n, uint16_t* XP,
                               int64_t pstride, int tile_rows, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % 16 != 0 || tile_rows != kXN) return hipErrorInvalidValue;
  const int64_t nthr = (n * ld + 7) / 8;
  hipLaunchKernelGGL(split_planes_kernel, dim3((unsigned)((nthr + 255) / 256)), dim3(256), 0, st,
                     X, ld, r0, n, XP, pstride, tile_rows);
  return hipGetLastError();
}

}  // namespace vs
