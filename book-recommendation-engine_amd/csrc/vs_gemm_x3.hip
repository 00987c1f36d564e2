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
// with the same tolerance as the plain fp32 kernel.  The same kernel body with
// two planes (hi, mid: products hh, hm, mh) is the filter pass of the
// filter-and-verify engine (gemm_topk_x2f; bound and verification further down).
//
// The exact engine splits INSIDE the kernel, from fp32 data: three pre-split
// planes are 6 B per element against 4 B of fp32, and the staging instructions,
// not the matrix cores, bound the first version of this engine, which streamed
// planes through LDS-DMA (profiles/r01_x3_probes.txt: no staging loads 359 ms,
// all of them 536 ms, every load an L2 hit 511 ms).  The filter pass can do
// either (template XD): split in-kernel from the blocked fp32 rows (XD = 0), or
// stream two pre-split planes — still 4 B per element — by LDS-DMA straight into
// the stage's LDS image, with no split VALU and no ds_write (XD = 1,
// split_rows_kernel builds them).
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
#include <climits>
#include <cmath>
#include <cstdlib>

#include "vs_device.h"

// Diagnostic builds only (tools/x3_probe.sh; timing only, results are wrong):
// 2 = no global loads in the K loop, 9 = three of the six products.
#ifndef VS_X3_PROBE
#define VS_X3_PROBE 0
#endif
#ifndef VS_X2F_PRIO
#define VS_X2F_PRIO 1
#endif

namespace vs {

namespace {

constexpr int kT = 256;                   // database rows (and queries) per tile
constexpr int kKB = 16;                   // K elements per stage
constexpr int kChunkF = kT * kKB;         // floats per (tile, K-block) chunk: 4096
constexpr int kPlaneB = kT * 32;          // one bf16 plane of one stage: 8 KB
constexpr int kSparkB = 8 * 16 * 64 * 4;  // epilogue parking, 4 KB per wave
constexpr int kNBuf = 2;                  // LDS images (stages in flight)
// NP planes per operand: 3 = exact split, 2 = hi/mid only (the filter pass)
template <int NP>
constexpr int lds_bytes() { return kNBuf * NP * kPlaneB + kSparkB; }
constexpr int kX3ChunkTiles = 16;         // database tiles per workgroup per launch

// 32-B LDS rows hold 2 chunks of 16 B; chunk c of row r is stored at
// c ^ (((r >> 3) ^ (r >> 2)) & 1).  Reads: each 16-lane ds_read_b128 group of the
// 32-row fragment reads (rows {0-3,12-15,20-27} / {4-11,16-19,28-31}, 256-B bank
// period) lands on 16 distinct 16-B slots; writes: each 8-lane ds_write_b128
// group (rows 8j..8j+7, 128-B bank period) covers 8 distinct slots, so neither
// conflicts.  (VS_X2F_SWZ=0 selects the older c ^ ((r >> 3) & 1): conflict-free
// reads, 2-way conflicted writes.)
#ifndef VS_X2F_SWZ
#define VS_X2F_SWZ 1
#endif
__device__ __forceinline__ int swz32(int r, int c) {
  return VS_X2F_SWZ ? c ^ (((r >> 3) ^ (r >> 2)) & 1) : c ^ ((r >> 3) & 1);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t cvt_pk(float a, float b) {  // v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
__device__ __forceinline__ float bf16_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf16_hi(uint32_t u) { return __uint_as_float(u & 0xFFFF0000u); }

// Splits 8 floats (two 16-B pieces) into the first NP planes of 8 bf16 (16 B
// each): hi, mid, lo.
template <int NP>
__device__ __forceinline__ void split_planes(const f32x4& a, const f32x4& b, uint4 (&pl)[NP]) {
  const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  uint32_t w[3][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x0 = v[2 * i], x1 = v[2 * i + 1];
    w[0][i] = cvt_pk(x0, x1);
    const float r0 = x0 - bf16_lo(w[0][i]), r1 = x1 - bf16_hi(w[0][i]);
    w[1][i] = cvt_pk(r0, r1);
    if constexpr (NP == 3) {
      const float s0 = r0 - bf16_lo(w[1][i]), s1 = r1 - bf16_hi(w[1][i]);
      w[2][i] = cvt_pk(s0, s1);
    }
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) pl[p] = make_uint4(w[p][0], w[p][1], w[p][2], w[p][3]);
}

// Publishes this wave's LDS writes and waits for every wave: raw s_barrier (no
// fence, so the global loads in flight are not drained).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ bf16x8 as_bf(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }

// LDS-DMA of 16 B per lane into the wave-uniform LDS byte address `lds`; M0 is
// written and restored inside the statement.  hipcc does not count it: the caller
// retires it with its own vmcnt.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}
// A 16-B register load hipcc does not count either; its destination is read only
// after a wait statement that names it "+v" (cdna_hip_programming.md §5.7).
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(const void* p) {
  u32x4 v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return __builtin_bit_cast(uint4, v);
}
// Ties a 16-B register value to the wait statement (a native vector, so the
// operand is a VGPR quad rather than an indirect struct).
#define VS_TIE16(q) "+v"(*reinterpret_cast<u32x4*>(&(q)))

}  // namespace

template <int KR, int MODE, int NP, int XD>
__device__ __forceinline__ void topk_body(
    const float* __restrict__ XB, const float* __restrict__ xaux, const uint4* __restrict__ QP,
    const float* __restrict__ qaux, int nqa, int nkb, int ntotal, int ntiles, int nsplit, int nqt,
    int64_t self0, int chunk, int nchunk, int KP, float* __restrict__ pkey,
    int* __restrict__ pid) {
  extern __shared__ __attribute__((aligned(16))) char smem[];  // lds_bytes<NP>()
  constexpr int kStageB = NP * kPlaneB;  // one LDS image: NP planes of one K-block

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
    auto load_q = [&](int kb, uint4 (&q)[NP]) {
      const uint4* p = qsrc + (int64_t)kb * 512;
#pragma unroll
      for (int j = 0; j < NP; ++j) q[j] = p[j * qpl];
    };
    auto write_x = [&](int buf, const f32x4& r0, const f32x4& r1) {
      uint4 pl[NP];
      split_planes<NP>(r0, r1, pl);
      char* base = smem + buf * kStageB + woff;
#pragma unroll
      for (int j = 0; j < NP; ++j) *(uint4*)(base + j * kPlaneB) = pl[j];
    };

    // The MFMAs of one stage over the image of `buf` with query planes qc.
    auto mma = [&](f32x16 (&acc)[8], int buf, const uint4 (&qc)[NP]) {
      const char* cb = smem + buf * kStageB + roff;
      uint4 x[NP];
#pragma unroll
      for (int j = 0; j < NP; ++j) x[j] = *(const uint4*)(cb + j * kPlaneB);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const char* nb = cb + (i + 1) * 32 * 32;
        f32x16 a = acc[i];
        // the products x_j q_l with j + l < NP (all six above 2^-24 for the exact
        // split; hh, hm, mh for the filter); each fragment register is refilled
        // with the next row block's fragment right after its last use
#pragma unroll
        for (int j = 0; j < NP; ++j) {
#pragma unroll
          for (int l = 0; l + j < NP; ++l)
            if (VS_X3_PROBE != 9 || j + l < 2)
              a = __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(x[j]), as_bf(qc[l]), a, 0, 0, 0);
          if (i < 7) x[j] = *(const uint4*)(nb + j * kPlaneB);
        }
        acc[i] = a;
      }
    };

    // One stage, XD = 0: MFMAs over the image of `buf` with query planes qc,
    // while stage+1's query planes load into qn, stage+2's database slice into
    // xn*, and stage+1's database slice (xc*) is split into the other image.
    auto stage = [&](f32x16 (&acc)[8], int buf, int kb_next, const uint4 (&qc)[NP],
                     uint4 (&qn)[NP], const f32x4& xc0, const f32x4& xc1, f32x4& xn0,
                     f32x4& xn1) {
      lds_barrier();  // this stage's image is complete; the previous one is free
      if (VS_X3_PROBE != 2) {
        load_q(kb_next, qn);
        load_x(xn0, xn1);
      }
      mma(acc, buf, qc);
      write_x(buf ^ 1, xc0, xc1);
    };

    // XD = 1.  Piece v (0 .. 8*NP-1) of a stage's image = plane v/8, rows
    // 32*(v%8) .. +31 (1 KiB); wave w moves pieces NP*w .. NP*w + NP-1.  Lane l
    // lands at bytes [16l, 16l+16) of its piece: row 32*(v%8) + l/2, 16-B slot
    // l&1, which must hold chunk (l&1) ^ ((row >> 3) & 1) — the swizzle goes on
    // the SOURCE address (the LDS side of LDS-DMA is lane-linear).  Query planes
    // come by asm loads too; every load of a stage is retired by one vmcnt(0) at
    // its end (counted and uncounted loads in one loop mis-wait).
    const char* xpb = (const char*)XB;
    const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(smem);
    const int prow = lane >> 1;
    const uint32_t psrc = (uint32_t)(prow * 2 + swz32(prow, lane & 1)) * 16u;
    auto dma_x = [&](int buf) {  // the stage at the cursor into image `buf`
      const char* cbase = xpb + ((int64_t)min(lt, t1 - 1) * nkb + lst) * kStageB + psrc;
#pragma unroll
      for (int j = 0; j < NP; ++j) {
        const int v = w * NP + j;
        glds16(cbase + v * 1024,
               __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)(buf * kStageB + v * 1024)));
      }
      if (++lst == nkb) {
        lst = 0;
        ++lt;
      }
    };
    auto load_q_asm = [&](int kb, uint4 (&q)[NP]) {
      const uint4* p = qsrc + (int64_t)kb * 512;
#pragma unroll
      for (int j = 0; j < NP; ++j) q[j] = gload16(p + j * qpl);
    };
    auto wait_all = [&](uint4 (&q)[NP]) {  // this wave's DMA and query loads landed
      if constexpr (NP == 2)
        asm volatile("s_waitcnt vmcnt(0)" : VS_TIE16(q[0]), VS_TIE16(q[1])::"memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" : VS_TIE16(q[0]), VS_TIE16(q[1]), VS_TIE16(q[2])::"memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    auto stage_dma = [&](f32x16 (&acc)[8], int buf, int kb_next, const uint4 (&qc)[NP],
                         uint4 (&qn)[NP]) {
      lds_barrier();  // this stage's image is complete; the previous one is free
      load_q_asm(kb_next, qn);
      dma_x(buf ^ 1);
      mma(acc, buf, qc);
      wait_all(qn);
    };

    uint4 qpa[NP], qpb[NP];    // query planes, two stages
    f32x4 xa0, xa1, xb0, xb1;  // raw database slices, two stages (XD = 0)
    if constexpr (XD == 0) {
      // prologue: stage 0's image and query planes, stage 1's slice in flight
      f32x4 x00, x01;
      load_x(x00, x01);
      load_q(0, qpa);
      load_x(xa0, xa1);
      write_x(0, x00, x01);
    } else {
      dma_x(0);
      load_q_asm(0, qpa);
      wait_all(qpa);
    }

    // waves 4-7 share their SIMDs with waves 0-3 and lose every VALU
    // arbitration on age; one static priority for that half (MI355X_MICROARCH.md,
    // "Two waves per SIMD" item 4)
    if (VS_X2F_PRIO && w >= 4) __builtin_amdgcn_s_setprio(1);
    float* spark = (float*)(smem + kNBuf * kStageB) + w * 16 * 64;

    // Epilogue of tile t (one 32-row block at a time): keys, a 16-bit candidate
    // mask against the lane's current worst entry, and insertion of the flagged
    // values only (after the first tiles almost nothing passes).
    auto epilogue = [&](const f32x16 (&acc)[8], int t) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r0 = t * kT + 32 * i;
        f32x4 xa[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          xa[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
          if constexpr (MODE == MODE_L2 || MODE == MODE_COS)
            xa[jj] = *(const f32x4*)(xaux + r0 + 8 * jj + 4 * h);
        }
        const float tk = lk[KR - 1];
        const int ti = li[KR - 1];
        uint32_t m = 0;
        f32x16 v16 = acc[i];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int rb = r0 + 8 * jj + 4 * h;
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
            const int row = r0 + (bi & 3) + 8 * (bi >> 2) + 4 * h;
            list_insert<KR, int>(lk, li, spark[bi * 64 + lane], row);
          } while (m);
        }
      }
    };

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
        if constexpr (XD == 0) {
          stage(acc, 0, k1, qpa, qpb, xa0, xa1, xb0, xb1);
          stage(acc, 1, k2, qpb, qpa, xb0, xb1, xa0, xa1);
        } else {
          stage_dma(acc, 0, k1, qpa, qpb);
          stage_dma(acc, 1, k2, qpb, qpa);
        }
      }
      epilogue(acc, t);
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

// The exact engine (three planes, six products) and the filter pass of bf16x2v
// (two planes, three products), named apart so that profiles tell them apart.
template <int KR, int MODE>
__global__ __launch_bounds__(512, 1) void gemm_topk_x3(
    const float* __restrict__ XB, const float* __restrict__ xaux, const uint4* __restrict__ QP,
    const float* __restrict__ qaux, int nqa, int nkb, int ntotal, int ntiles, int nsplit, int nqt,
    int64_t self0, int chunk, int nchunk, int KP, float* __restrict__ pkey,
    int* __restrict__ pid) {
  topk_body<KR, MODE, 3, 0>(XB, xaux, QP, qaux, nqa, nkb, ntotal, ntiles, nsplit, nqt, self0,
                            chunk, nchunk, KP, pkey, pid);
}
// XD: database operand from the blocked fp32 rows (0) or from pre-split planes
// by LDS-DMA (1).
template <int KR, int MODE, int XD>
__global__ __launch_bounds__(512, 1) void gemm_topk_x2f(
    const float* __restrict__ XB, const float* __restrict__ xaux, const uint4* __restrict__ QP,
    const float* __restrict__ qaux, int nqa, int nkb, int ntotal, int ntiles, int nsplit, int nqt,
    int64_t self0, int chunk, int nchunk, int KP, float* __restrict__ pkey,
    int* __restrict__ pid) {
  topk_body<KR, MODE, 2, XD>(XB, xaux, QP, qaux, nqa, nkb, ntotal, ntiles, nsplit, nqt, self0,
                             chunk, nchunk, KP, pkey, pid);
}

template <int KR, int MODE, int NP, int XD>
static const void* x3_kernel() {
  if constexpr (NP == 3) return (const void*)gemm_topk_x3<KR, MODE>;
  else return (const void*)gemm_topk_x2f<KR, MODE, XD>;
}

template <int KR, int MODE, int NP, int XD>
static hipError_t x3_launch(const X3Args& a, Partials part, hipStream_t st, int* ndispatch) {
  constexpr int lds = lds_bytes<NP>();
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute(x3_kernel<KR, MODE, NP, XD>(),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
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
    const int nkb = (int)(a.ld / kKB);
    if constexpr (NP == 3)
      hipLaunchKernelGGL((gemm_topk_x3<KR, MODE>), dim3(nqt * a.nsplit), dim3(512),
                         lds, st, a.XB, a.xaux, a.QP, a.qaux, a.nqa, nkb, a.ntotal,
                         ntiles, a.nsplit, nqt, a.self0, c, nchunk, part.KP, part.key, part.id);
    else
      hipLaunchKernelGGL((gemm_topk_x2f<KR, MODE, XD>), dim3(nqt * a.nsplit), dim3(512),
                         lds, st, a.XB, a.xaux, a.QP, a.qaux, a.nqa, nkb, a.ntotal,
                         ntiles, a.nsplit, nqt, a.self0, c, nchunk, part.KP, part.key, part.id);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (ndispatch) *ndispatch = nchunk;
  return hipSuccess;
}

// Exact split (NP = 3, XD = 0): every list length, IP / L2 / COS.  Filter pass
// (NP = 2): IP and L2 with the list lengths x2f_list_len returns, from blocked
// fp32 rows (XD = 0) or pre-split planes (XD = 1).
template <int KR>
static hipError_t x3_dispatch(int mode, int np, int xd, const X3Args& a, Partials part,
                              hipStream_t st, int* ndispatch) {
  if (np == 3 && xd == 0 && KR <= 24) {
    switch (mode) {
      case MODE_IP:
        return x3_launch<KR, MODE_IP, 3, 0>(a, part, st, ndispatch);
      case MODE_L2:
        return x3_launch<KR, MODE_L2, 3, 0>(a, part, st, ndispatch);
      case MODE_COS:
        return x3_launch<KR, MODE_COS, 3, 0>(a, part, st, ndispatch);
      default:
        return hipErrorInvalidValue;
    }
  }
  if constexpr (KR == 12 || KR == 16 || KR == 32) {
    if (np == 2 && mode == MODE_IP)
      return xd ? x3_launch<KR, MODE_IP, 2, 1>(a, part, st, ndispatch)
                : x3_launch<KR, MODE_IP, 2, 0>(a, part, st, ndispatch);
    if (np == 2 && mode == MODE_L2)
      return xd ? x3_launch<KR, MODE_L2, 2, 1>(a, part, st, ndispatch)
                : x3_launch<KR, MODE_L2, 2, 0>(a, part, st, ndispatch);
    if (np == 2 && mode == MODE_COS && xd == 0 && KR == 16)
      return x3_launch<KR, MODE_COS, 2, 0>(a, part, st, ndispatch);
  }
  return hipErrorInvalidValue;
}

// Longer lists do not fit the register file beside the 128 accumulators (KR=32
// spills ~100 registers into the K loop of the exact split): those searches take
// the fp32 engine.
int x3_list_len(int need) {
  return need <= 8 ? 8 : need <= 12 ? 12 : need <= 16 ? 16 : need <= 20 ? 20 : need <= 24 ? 24 : 0;
}

// Filter pass: number of merged approximate candidates for `need` exact entries,
// a margin of at least 8 beyond the entries the merge needs (0 = unsupported).
int x2f_list_len(int need) {
  return need + 8 <= 24 ? 24 : need + 8 <= 32 ? 32 : need + 8 <= 64 ? 64 : 0;
}

// Per-lane list length of the filter pass.  A lane list does not have to hold
// all KF candidates: a full list's last entry bounds every row the lane dropped,
// and the verification takes the smallest such floor into its condition (see
// below).  16 entries keep the kernel's 256 registers free of spills (32 spill);
// on uncorrelated data each lane list sees 1/P of the rows, so its 16th entry
// sits near rank 16·P overall, far behind the KF-th.  VS_X2F_L=12 / 32 override.
int x2f_lane_len() {
  const char* e = getenv("VS_X2F_L");
  const int v = e ? atoi(e) : 0;
  return v == 12 || v == 32 ? v : 16;
}

hipError_t launch_gemm_topk_x3(int KR, int mode, int np, int xd, const X3Args& a, Partials part,
                               hipStream_t st, int* ndispatch) {
  // ld % 32: an even number of K-blocks per tile keeps the LDS image parity of a
  // stage equal to its K-block parity across tiles
  if (a.nq_pad % kT != 0 || a.ld % (2 * kKB) != 0 || KR > part.KP || part.P != 2 * a.nsplit ||
      a.nsplit < 1 || (np != 2 && np != 3) || (xd != 0 && xd != 1))
    return hipErrorInvalidValue;
  switch (KR) {
    case 8:
      return x3_dispatch<8>(mode, np, xd, a, part, st, ndispatch);
    case 12:
      return x3_dispatch<12>(mode, np, xd, a, part, st, ndispatch);
    case 16:
      return x3_dispatch<16>(mode, np, xd, a, part, st, ndispatch);
    case 20:
      return x3_dispatch<20>(mode, np, xd, a, part, st, ndispatch);
    case 24:
      return x3_dispatch<24>(mode, np, xd, a, part, st, ndispatch);
    case 32:
      return x3_dispatch<32>(mode, np, xd, a, part, st, ndispatch);
    default:
      return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// Filter-and-verify (engine VS_ENGINE_BF16X2_VERIFY).  The NP = 2 pass scores
// every row with hh + hm + mh; the dropped terms and the fp32 accumulation are
// bounded by  |approx_key - exact_key| <= Bkey  (from coef * |x| * |q|, coef =
// x2f_bound_coef).  Let a = the sorted approximate keys of the KF best
// candidates of a query and E = their exact keys, sorted; the M-th entry E[M-1]
// bounds the true M-th best exact key from above (M candidates reach it).  Every
// row outside the candidate set has approx key >= a[KF-1], so exact key >=
// a[KF-1] - Bkey; whenever
//     a[KF-1] - Bkey > E[M-1]
// those rows are strictly worse than the true M-th entry, and the exact top-M
// (ties included) is E's first M entries.  verify_rescore_kernel rescores the
// candidates exactly (fp64 accumulation of the fp32 products, rounded to fp32),
// sorts them and checks the condition; queries that fail it are flagged for
// the exact engine.

// Bound coefficient for `ld` K elements: the three dropped product classes of
// each term (hl, lh, mm: <= 3 * 2^-16 (1 + 2^-8)^2 |x_k q_k|, the rest < 2^-23),
// plus the accumulation of 3*ld products whose every step may be off by one
// ulp (u = 2^-23, which also covers truncating adders):
// gamma = n u / (1 - n u) on sum |products| <= 1.0235 sum |x_k q_k| <= 1.0235 |x||q|.
double x2f_bound_coef(int64_t ld) {
  const double u = std::ldexp(1.0, -23);
  const double n = 3.0 * (double)ld + 1.0;
  const double gamma = n * u / (1.0 - n * u);
  const double drop = 3.0 * std::ldexp(1.0, -16) * (1.0 + std::ldexp(1.0, -8)) *
                          (1.0 + std::ldexp(1.0, -8)) +
                      std::ldexp(1.0, -23);
  return (drop + gamma * 1.0235) * (1.0 + 1e-6);
}

// Cosine keys -(s * qinv * xinv), qinv/xinv = 1/sqrt of the stored squared norms
// (those norms carry up to gamma(ld) relative error, so |q| * qinv <= 1 + 1.1 gamma):
// |key_a - key_e| <= coef |q||x| qinv xinv (1 + u) + two roundings of |key| <~ 1,
// i.e. <= (coef + 2^-22)(1 + 3 gamma(ld)), independent of the rows.
double x2f_cos_key_bound(int64_t ld) {
  const double u = std::ldexp(1.0, -23);
  const double n = (double)ld;
  const double gamma = n * u / (1.0 - n * u);
  return (x2f_bound_coef(ld) + std::ldexp(1.0, -22)) * (1.0 + 3.0 * gamma) * (1.0 + 1e-6);
}

__global__ __launch_bounds__(256) void max_norm_kernel(const float* __restrict__ norms, int64_t n,
                                                       unsigned* __restrict__ out) {
  unsigned m = 0;  // non-negative floats (and NaN, above them) order as their bits
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = max(m, __float_as_uint(norms[i]) & 0x7FFFFFFFu);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned)__shfl_xor((int)m, o));
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

hipError_t launch_max_norm(const float* norms, int64_t n, unsigned* out, hipStream_t st) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(unsigned), st);
  if (e != hipSuccess || n <= 0) return e;
  const int64_t blocks = std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(max_norm_kernel, dim3((unsigned)blocks), dim3(256), 0, st, norms, n, out);
  return hipGetLastError();
}

// One wave per query.  Dk/Ik: the KF best approximate keys (ascending) and local
// rows of each query; X/xn: fp32 rows (stride ld) and squared norms; Q/qn: query
// rows and squared norms.  Writes a sorted list of KF exact (key, row) entries,
// padded to KP, and fail[q].
template <int MODE>
__global__ __launch_bounds__(64) void verify_rescore_kernel(
    int KF, int M, const float* __restrict__ Dk, const int64_t* __restrict__ Ik,
    const float* __restrict__ X, const float* __restrict__ xn, const float* __restrict__ Q,
    const float* __restrict__ qn, int64_t ld, double coef, const unsigned* __restrict__ xmax2,
    const float* __restrict__ lkey, const int* __restrict__ lid, int P, int LKP, int L,
    float* __restrict__ okey, int* __restrict__ oid, int KP, int* __restrict__ fail,
    const float* __restrict__ qinv, const float* __restrict__ xinv) {
  __shared__ float ek[64];
  const int lane = threadIdx.x;
  const int q = blockIdx.x;
  const float a = lane < KF ? Dk[(int64_t)q * KF + lane] : FLT_MAX;
  const int id = lane < KF ? (int)Ik[(int64_t)q * KF + lane] : -1;
  const float aK = __shfl(a, KF - 1);
  const int idK = __shfl(id, KF - 1);
  // T: the KF-th merged key (if the merge found KF) and the last key of every
  // full lane list; `bounded` = false when neither exists (the candidates are
  // every admissible row)
  bool bounded = idK >= 0;
  float T = idK >= 0 ? aK : FLT_MAX;
  for (int j = lane; j < P; j += 64) {
    const int64_t o = ((int64_t)q * P + j) * LKP + L - 1;
    if (lid[o] >= 0) {
      bounded = true;
      T = fminf(T, lkey[o]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) T = fminf(T, __shfl_xor(T, o));
  bounded = __any(bounded);

  // exact keys, one candidate at a time across the wave
  const float* qrow = Q + (int64_t)q * ld;
  for (int j = 0; j < KF; ++j) {
    const int r = __shfl(id, j);
    if (r < 0) {
      if (lane == 0) ek[j] = FLT_MAX;
      continue;
    }
    const float* xr = X + (int64_t)r * ld;
    double acc = 0.0;
    for (int64_t c = lane * 4; c < ld; c += 256) {
      const f32x4 xv = *(const f32x4*)(xr + c);
      const f32x4 qv = *(const f32x4*)(qrow + c);
      acc = fma((double)xv.x, (double)qv.x, acc);
      acc = fma((double)xv.y, (double)qv.y, acc);
      acc = fma((double)xv.z, (double)qv.z, acc);
      acc = fma((double)xv.w, (double)qv.w, acc);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
      const float ip = (float)acc;
      // the filter epilogue's key formulas (topk_body), on the exact dot product
      ek[j] = MODE == MODE_L2    ? l2_from_ip(qn[q], xn[r], ip)
              : MODE == MODE_COS ? -(ip * (qinv[q] * xinv[r]))
                                 : -ip;
    }
  }
  __syncthreads();
  // rank sort of (key, row); empty slots last, in lane order among themselves
  const float k0 = lane < KF ? ek[lane] : FLT_MAX;
  const int i0 = id < 0 ? INT_MAX : id;
  int rank = 0;
  for (int j = 0; j < KF; ++j) {
    const float kj = __shfl(k0, j);
    const int ij = __shfl(i0, j);
    rank += (lex_less(kj, ij, k0, i0) || (kj == k0 && ij == i0 && j < lane)) ? 1 : 0;
  }
  float* ok = okey + (int64_t)q * KP;
  int* oi = oid + (int64_t)q * KP;
  if (lane < KF) {
    ok[rank] = k0;
    oi[rank] = id;  // -1 for empty slots
  } else if (lane < KP) {
    ok[lane] = FLT_MAX;
    oi[lane] = -1;
  }
  // the M-th exact key (the lane whose rank is M-1 publishes it)
  if (lane < KF && rank == M - 1) ek[63] = k0;
  __syncthreads();
  const float eM = ek[63];
  const double qn2 = (double)qn[q];
  const double xm2 = (double)__uint_as_float(*xmax2);
  double bkey = coef * sqrt(qn2) * sqrt(xm2);
  if constexpr (MODE == MODE_L2)  // key = (|q|^2 + |x|^2) - 2 ip, each side rounded
    bkey = 2.0 * bkey + 8.0 * std::ldexp(1.0, -24) * (qn2 + xm2);
  if constexpr (MODE == MODE_COS)  // scale-free: the host passes the whole key bound
    bkey = coef;
  const bool pass = !bounded || ((double)T - bkey > (double)eM && isfinite(T) && isfinite(eM) &&
                                  isfinite(bkey));
  if (lane == 0) fail[q] = pass ? 0 : 1;
}

hipError_t launch_verify_rescore(int mode, int nq, int KF, int M, const float* Dk,
                                 const int64_t* Ik, const float* X, const float* xn,
                                 const float* Q, const float* qn, int64_t ld, double coef,
                                 const unsigned* xmax2, Partials lists, int L, float* okey,
                                 int* oid, int KP, int* fail, hipStream_t st, const float* qinv,
                                 const float* xinv) {
  if (KF > 64 || KP > 64 || KF > KP || M < 1 || M > KF || ld % 4 != 0 || L < 1 ||
      L > lists.KP)
    return hipErrorInvalidValue;
  if (nq <= 0) return hipSuccess;
  if (mode == MODE_IP)
    hipLaunchKernelGGL(verify_rescore_kernel<MODE_IP>, dim3(nq), dim3(64), 0, st, KF, M, Dk, Ik,
                       X, xn, Q, qn, ld, coef, xmax2, lists.key, lists.id, lists.P, lists.KP, L,
                       okey, oid, KP, fail, qinv, xinv);
  else if (mode == MODE_L2)
    hipLaunchKernelGGL(verify_rescore_kernel<MODE_L2>, dim3(nq), dim3(64), 0, st, KF, M, Dk, Ik,
                       X, xn, Q, qn, ld, coef, xmax2, lists.key, lists.id, lists.P, lists.KP, L,
                       okey, oid, KP, fail, qinv, xinv);
  else if (mode == MODE_COS && qinv && xinv)
    hipLaunchKernelGGL(verify_rescore_kernel<MODE_COS>, dim3(nq), dim3(64), 0, st, KF, M, Dk, Ik,
                       X, xn, Q, qn, ld, coef, xmax2, lists.key, lists.id, lists.P, lists.KP, L,
                       okey, oid, KP, fail, qinv, xinv);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Wide verification of a flagged query (one 256-thread workgroup each).  The
// condition above only needs a threshold T such that every row outside the
// rescored set has approximate key >= T: the smallest last entry of the full lane
// lists is one (a full list dropped only rows lexicographically after its last
// entry), and then the set may be *all* list entries below T, not just the KF
// merged ones.  Each of the P lists sees 1/P of the rows, so its 16th entry sits
// near overall rank 16·P and T, their minimum, a few hundred rows deep (C3: P =
// 32), far behind the KF-th; queries whose best keys crowd within
// the bound (near-duplicates, clustered embeddings) are settled here without a
// second pass over the corpus.  More than kWideCap entries below T, fewer than M,
// or a non-finite key: the query stays flagged.
template <int MODE>
__global__ __launch_bounds__(256) void verify_wide_kernel(
    const int* __restrict__ qlist, int KF, int M, const float* __restrict__ X,
    const float* __restrict__ xn, const float* __restrict__ Q, const float* __restrict__ qn,
    int64_t ld, double coef, const unsigned* __restrict__ xmax2, const float* __restrict__ lkey,
    const int* __restrict__ lid, int P, int LKP, int L, float* __restrict__ okey,
    int* __restrict__ oid, int KP, int* __restrict__ fail, const float* __restrict__ qinv,
    const float* __restrict__ xinv) {
  __shared__ float ck[kWideCap];
  __shared__ int cid[kWideCap];
  __shared__ float wT[4];
  __shared__ int wB[4];
  __shared__ int cnt, bad;
  __shared__ float eMs;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int q = qlist[blockIdx.x];
  const int64_t lbase = (int64_t)q * P * LKP;
  float T = FLT_MAX;
  bool bounded = false;
  for (int j = tid; j < P; j += 256) {
    const int64_t o = lbase + (int64_t)j * LKP + L - 1;
    if (lid[o] >= 0) {
      bounded = true;
      T = fminf(T, lkey[o]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) T = fminf(T, __shfl_xor(T, o));
  bounded = __any(bounded);
  if (lane == 0) {
    wT[wv] = T;
    wB[wv] = bounded ? 1 : 0;
  }
  if (tid == 0) {
    cnt = 0;
    bad = 0;
    eMs = FLT_MAX;
  }
  __syncthreads();
  T = fminf(fminf(wT[0], wT[1]), fminf(wT[2], wT[3]));
  bounded = (wB[0] | wB[1] | wB[2] | wB[3]) != 0;
  // gather every entry below T (all entries when no list is full)
  for (int j = tid; j < P * L; j += 256) {
    const int64_t o = lbase + (int64_t)(j / L) * LKP + j % L;
    const int r = lid[o];
    if (r >= 0 && (!bounded || lkey[o] < T)) {
      const int s = atomicAdd(&cnt, 1);
      if (s < kWideCap) cid[s] = r;
    }
  }
  __syncthreads();
  const int n = cnt;
  if (n > kWideCap || n < M || !isfinite(T)) return;  // uniform: stays flagged
  // exact keys, one candidate per wave at a time (fp64 accumulation, as above)
  const float* qrow = Q + (int64_t)q * ld;
  for (int j = wv; j < n; j += 4) {
    const int r = cid[j];
    const float* xr = X + (int64_t)r * ld;
    double acc = 0.0;
    for (int64_t c = lane * 4; c < ld; c += 256) {
      const f32x4 xv = *(const f32x4*)(xr + c);
      const f32x4 qv = *(const f32x4*)(qrow + c);
      acc = fma((double)xv.x, (double)qv.x, acc);
      acc = fma((double)xv.y, (double)qv.y, acc);
      acc = fma((double)xv.z, (double)qv.z, acc);
      acc = fma((double)xv.w, (double)qv.w, acc);
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
      const float ip = (float)acc;
      const float key = MODE == MODE_L2    ? l2_from_ip(qn[q], xn[r], ip)
                        : MODE == MODE_COS ? -(ip * (qinv[q] * xinv[r]))
                                           : -ip;
      ck[j] = key;
      if (!isfinite(key)) bad = 1;
    }
  }
  __syncthreads();
  if (bad) return;  // uniform
  // rank of each (key, row) among the n (rows are distinct: the lists are disjoint)
  float* ok = okey + (int64_t)q * KP;
  int* oi = oid + (int64_t)q * KP;
  for (int j = tid; j < n; j += 256) {
    const float kj = ck[j];
    const int ij = cid[j];
    int rank = 0;
    for (int t = 0; t < n; ++t) rank += lex_less(ck[t], cid[t], kj, ij) ? 1 : 0;
    if (rank < KF) {
      ok[rank] = kj;
      oi[rank] = ij;
    }
    if (rank == M - 1) eMs = kj;
  }
  for (int j = min(n, KF) + tid; j < KP; j += 256) {
    ok[j] = FLT_MAX;
    oi[j] = -1;
  }
  __syncthreads();
  const float eM = eMs;
  const double qn2 = (double)qn[q];
  const double xm2 = (double)__uint_as_float(*xmax2);
  double bkey = coef * sqrt(qn2) * sqrt(xm2);
  if constexpr (MODE == MODE_L2) bkey = 2.0 * bkey + 8.0 * std::ldexp(1.0, -24) * (qn2 + xm2);
  if constexpr (MODE == MODE_COS) bkey = coef;
  const bool pass = !bounded || ((double)T - bkey > (double)eM && isfinite(eM) && isfinite(bkey));
  if (tid == 0 && pass) fail[q] = 0;
}

hipError_t launch_verify_wide(int mode, int nf, const int* qlist, int KF, int M, const float* X,
                              const float* xn, const float* Q, const float* qn, int64_t ld,
                              double coef, const unsigned* xmax2, Partials lists, int L,
                              float* okey, int* oid, int KP, int* fail, hipStream_t st,
                              const float* qinv, const float* xinv) {
  if (KF > KP || M < 1 || M > KF || ld % 4 != 0 || L < 1 || L > lists.KP) return hipErrorInvalidValue;
  if (nf <= 0) return hipSuccess;
#define VS_WIDE(MD)                                                                            \
  hipLaunchKernelGGL(verify_wide_kernel<MD>, dim3(nf), dim3(256), 0, st, qlist, KF, M, X, xn, Q, \
                     qn, ld, coef, xmax2, lists.key, lists.id, lists.P, lists.KP, L, okey, oid,  \
                     KP, fail, qinv, xinv)
  if (mode == MODE_IP)
    VS_WIDE(MODE_IP);
  else if (mode == MODE_L2)
    VS_WIDE(MODE_L2);
  else if (mode == MODE_COS && qinv && xinv)
    VS_WIDE(MODE_COS);
  else
    return hipErrorInvalidValue;
#undef VS_WIDE
  return hipGetLastError();
}

// Splits fp32 query rows [0, n) (stride ld) into the first NP bf16 planes of the
// MFMA B fragments: uint4 ((p*nqt + r/256)*nkb + kb)*512 + ((r%256)/32)*64 + lane,
// lane = h*32 + r%32, holding k = 16kb + {4h..4h+3, 8+4h..8+4h+3} (the K
// permutation of the blocked database rows).  One thread per (row, kb, h).
template <int NP>
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
  uint4 v[NP];
  split_planes<NP>(a, c, v);
  const int64_t o = ((r / kT) * nkb + kb) * 512 + ((r % kT) / 32) * 64 + hh * 32 + r % 32;
  const int64_t pl = (int64_t)nqt * nkb * 512;
#pragma unroll
  for (int j = 0; j < NP; ++j) QP[o + j * pl] = v[j];
}

hipError_t launch_split_queries(const float* Q, int64_t ld, int64_t n, int nq_pad, int np,
                                uint4* QP, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % kKB != 0 || nq_pad % kT != 0 || n > nq_pad || (np != 2 && np != 3))
    return hipErrorInvalidValue;
  const int64_t items = n * (ld / kKB) * 2;
  const dim3 grid((unsigned)((items + 255) / 256));
  if (np == 3)
    hipLaunchKernelGGL(split_queries_kernel<3>, grid, dim3(256), 0, st, Q, ld, n, nq_pad / kT, QP);
  else
    hipLaunchKernelGGL(split_queries_kernel<2>, grid, dim3(256), 0, st, Q, ld, n, nq_pad / kT, QP);
  return hipGetLastError();
}

// Splits fp32 database rows [r0, r0+n) into NP bf16 planes laid out as the LDS
// images of the stages (XD = 1): chunk (t, kb) holds NP planes of 8 KB, and 16-B
// chunk h (k = 16kb + {4h..4h+3, 8+4h..8+4h+3}, the K permutation) of plane j,
// row r%256 is uint4 ((t*nkb + kb)*NP + j)*512 + (r%256)*2 + h (unswizzled; the
// kernel swizzles on the source address).  One thread per (row, kb, h).
template <int NP>
__global__ __launch_bounds__(256) void split_rows_kernel(const float* __restrict__ X, int64_t ld,
                                                         int64_t r0, int64_t n,
                                                         uint4* __restrict__ XP) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nkb = ld / kKB;
  if (p >= n * nkb * 2) return;
  const int64_t r = r0 + p / (nkb * 2);
  const int64_t kb = (p / 2) % nkb;
  const int hh = (int)(p & 1);
  const float* src = X + r * ld + kb * kKB + 4 * hh;
  const f32x4 a = *(const f32x4*)src;
  const f32x4 c = *(const f32x4*)(src + 8);
  uint4 v[NP];
  split_planes<NP>(a, c, v);
  const int64_t base = ((r / kT) * nkb + kb) * NP * 512 + (r % kT) * 2 + hh;
#pragma unroll
  for (int j = 0; j < NP; ++j) XP[base + j * 512] = v[j];
}

hipError_t launch_split_rows(const float* X, int64_t ld, int64_t r0, int64_t n, int np,
                             uint4* XP, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % kKB != 0 || (np != 2 && np != 3)) return hipErrorInvalidValue;
  const int64_t items = n * (ld / kKB) * 2;
  const dim3 grid((unsigned)((items + 255) / 256));
  if (np == 3)
    hipLaunchKernelGGL(split_rows_kernel<3>, grid, dim3(256), 0, st, X, ld, r0, n, XP);
  else
    hipLaunchKernelGGL(split_rows_kernel<2>, grid, dim3(256), 0, st, X, ld, r0, n, XP);
  return hipGetLastError();
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
