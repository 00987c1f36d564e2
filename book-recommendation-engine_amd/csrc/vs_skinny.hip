// vs_skinny.hip — small-batch (nq <= 32) fused distance + top-k, HBM-bound.
//
// Every database row is used once per launch: the corpus streams through LDS
// once (whole 128-B lines per row, the access pattern HBM wants) into 16x16 MFMA
// tiles whose N dimension is the (padded) query batch — v_mfma_f32_16x16x4_f32
// for fp32 rows, v_mfma_f32_16x16x32_bf16 for bf16 rows.  Padding the batch to 16
// costs MFMA cycles the memory system does not wait for (10M x 1536 x 16 queries
// is 0.49 TFLOP = 3 ms of fp32 matrix time against 9.6 ms of HBM time), and
// unlike a dot-product GEMV it needs no cross-lane reductions.
//
// Geometry (16x16 C/D layout: column = lane & 15, row = 4 * (lane >> 4) + reg):
//   A = 16 database rows, B = 16 queries.  A workgroup (4 waves) owns a tile of
//   128 rows (32 per wave = 2 row groups of 16) against all the batch's queries
//   and walks K in 128-B slices: LDS-DMA (global_load_lds_dwordx4) stages 8 rows
//   x 128 B per wave instruction (whole cache lines) into a ring of NB slice
//   images, NB - 1 slices in flight (two workgroups per CU: ~110 KB of loads in
//   flight per CU, what HBM needs at this latency; the round-2 form, 256-row
//   tiles double-buffered, held 64 KB and reached 0.78 of HBM at C5).  Fragments
//   are read from LDS with the same XOR swizzle as the GEMM (16-B chunk c of
//   row r at c ^ ((r >> 1) & 7): conflict-free ds_read_b128).  Per 64-B
//   k-chunk, lane l
//   takes the 16 B at chunk offset 16 * (l >> 4) of row l & 15 — of the X row for
//   A, of query row l & 15 for B.  fp32: the 4 floats feed 4 MFMAs (instruction t
//   uses element t, so lane group g covers k = 4g + t); bf16: the 8 bf16 are the
//   operand (k = 8g + j).  Each query fragment serves both row groups.
//   After the K loop lane l holds, for query l & 15 (+16 for the second query
//   group), the scores of rows rowbase + 16 * grp + 4 * (l >> 4) + reg: 4 lanes
//   share a query, each with its own register list; the block folds its 16
//   lists per query in LDS and emits one.
#include "vs_device.h"

namespace vs {

typedef float f32x4v __attribute__((ext_vector_type(4)));

// LDS-DMA of 16 B per lane into the wave-uniform LDS byte address `lds` (M0 set
// and restored inside the statement), from a uniform base plus a 32-bit lane
// offset.  hipcc does not count it: the K loop retires the slices with counted
// waits of its own (the builtin form would make hipcc drain vmcnt to 0 before
// every LDS read, i.e. one slice in flight).
__device__ __forceinline__ void skinny_glds(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// The same with the non-temporal cache policy: the plane passes stream every
// row piece once, from one CU (MI355X_MICROARCH.md "nt-weights": nt on a stream
// that ONE CU reads once).  C3 batch 1 over the int8 plane: 2.80 -> 2.58 ms per
// query, the pass 2.49 -> 2.29 ms = 0.77 -> 0.84 of HBM (profiles/r06snt, two
// rounds); the query pieces, which every CU reads, keep the default policy.
template <bool NT>
__device__ __forceinline__ void skinny_glds_p(const void* sbase, uint32_t voff, uint32_t lds) {
  if constexpr (!NT) {
    skinny_glds(sbase, voff, lds);
  } else {
    uint32_t keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds)
        : "memory");
  }
}

constexpr int kSkinnyRows = 128;  // database rows per tile (32 per wave)

// slice images in the ring: 4 for one query group (4 x 18 KB per workgroup),
// 3 for two (4 x 20 KB would not leave two workgroups per CU)
template <int NQG>
constexpr int skinny_nbuf() { return NQG == 1 ? 4 : 3; }

template <int KP, int MODE, typename T, int NQG>
__global__ __launch_bounds__(256, 2) void skinny_topk(const T* __restrict__ X,
                                                      const float* __restrict__ xaux,
                                                      const T* __restrict__ Q,
                                                      const float* __restrict__ qaux, int64_t ld,
                                                      int nq, int ntotal, int rows_per_block,
                                                      float* __restrict__ pkey,
                                                      int* __restrict__ pid,
                                                      const int* __restrict__ qcount) {
  static_assert(KP <= 32, "skinny path keeps at most 32 entries per list");
  // a gathered batch (the staged engine's last stage): nothing to do when the
  // device-side count is 0 (the lists are then never read)
  if (qcount && *qcount <= 0) return;  // uniform
  constexpr int NB = skinny_nbuf<NQG>();
  constexpr int R = kSkinnyRows;
  // LDS, three lives: [NB images][128 X rows + 16*NQG query rows][128 B] during
  // the K loop; per-thread key parking (8 x 256 floats) in the epilogue (every
  // slice retired by then); the per-query list fold ([16 queries][16 lists][KP]
  // keys + ids) at the end.
  constexpr int kRowsPerBuf = R + 16 * NQG;
  constexpr int kStageWords = NB * kRowsPerBuf * 32;
  constexpr int kFold = 16 * 16 * KP;
  constexpr int kWords0 = kStageWords > 2 * kFold ? kStageWords : 2 * kFold;
  constexpr int kWords = kWords0 > 8 * 256 ? kWords0 : 8 * 256;
  static_assert(2 * kWords * 4 <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) float lds[kWords];
  float* spark = lds;
  float* mk = lds;
  int* mi = (int*)(lds + kFold);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;  // lane group: 16-B offset inside a 64-B k-chunk
  const int c16 = lane & 15;
  const int nslice = (int)(ld * (int64_t)sizeof(T) / 128);
  const uint32_t ldb = (uint32_t)(ld * (int64_t)sizeof(T));
  const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(lds);

  float qa[NQG];
  int qcol[NQG];
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) {
    qcol[qg] = qg * 16 + c16;
    qa[qg] = 0.0f;
    if constexpr (MODE == MODE_L2) qa[qg] = qaux[qcol[qg]];
  }

  float lk[NQG][KP];
  int li[NQG][KP];
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) list_init<KP, int>(lk[qg], li[qg]);

  const int rb0 = blockIdx.x * rows_per_block;
  const int rb1 = min(rb0 + rows_per_block, (ntotal + 255) & ~255);
  // DMA geometry: lane L of a wave instruction moves 16 B of row (L >> 3) of an
  // 8-row group; the swizzle depends on the group only through its parity.
  const int srow = lane >> 3;
  uint32_t soff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int row = par * 8 + srow;
    soff[par] = (uint32_t)srow * ldb + (uint32_t)((lane & 7) ^ ((row >> 1) & 7)) * 16u;
  }
  const int fsw = (c16 >> 1) & 7;  // fragment rows 16*grp + c16 share (row >> 1) & 7
  // the query piece this wave stages per slice: 2 NQG pieces of 8 rows over the
  // 4 waves, every wave one (NQG = 1: two waves per piece, identical bytes to
  // identical LDS addresses), so every wave issues 5 loads per slice and one
  // counted wait serves all of them
  const int qpc = NQG == 1 ? (w & 1) : w;

  for (int tb = rb0; tb < rb1; tb += R) {
    f32x4v acc[NQG][2];
#pragma unroll
    for (int qg = 0; qg < NQG; ++qg)
#pragma unroll
      for (int grp = 0; grp < 2; ++grp) acc[qg][grp] = (f32x4v){0.f, 0.f, 0.f, 0.f};
    const char* xt = (const char*)(X + (int64_t)(tb + 32 * w) * ld);

    auto stage = [&](int sl) {
      const uint32_t base = lds0 + (uint32_t)((sl % NB) * kRowsPerBuf * 128);
      const char* xs = xt + sl * 128;
#pragma unroll
      for (int i = 0; i < 4; ++i)  // this wave's 32 rows
        skinny_glds(xs, soff[i & 1] + (uint32_t)(i * 8) * ldb,
                    __builtin_amdgcn_readfirstlane(base + (uint32_t)(32 * w + 8 * i) * 128u));
      skinny_glds((const char*)Q + sl * 128, soff[qpc & 1] + (uint32_t)(qpc * 8) * ldb,
                  __builtin_amdgcn_readfirstlane(base + (uint32_t)(R + 8 * qpc) * 128u));
    };

    // slices 0 .. NB-2 in flight, then retire slice 0
#pragma unroll
    for (int i = 0; i < NB - 1; ++i)
      if (i < nslice) stage(i);  // uniform
    if (nslice >= 3 && NB >= 4) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (nslice >= 2) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int sl = 0; sl < nslice; ++sl) {
      // slice sl+NB-1 into the image slice sl-1 used (every wave passed the
      // barrier after reading it)
      if (sl + NB - 1 < nslice) stage(sl + NB - 1);
      const float* cb = lds + (sl % NB) * kRowsPerBuf * 32;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int coff = ((4 * c + g) ^ fsw) * 4;  // in floats
        f32x4v qf[NQG];
#pragma unroll
        for (int qg = 0; qg < NQG; ++qg)
          qf[qg] = *(const f32x4v*)(cb + (R + 16 * qg + c16) * 32 + coff);
        f32x4v xf[2];
#pragma unroll
        for (int grp = 0; grp < 2; ++grp)
          xf[grp] = *(const f32x4v*)(cb + (32 * w + 16 * grp + c16) * 32 + coff);
#pragma unroll
        for (int qg = 0; qg < NQG; ++qg) {
#pragma unroll
          for (int grp = 0; grp < 2; ++grp) {
            if constexpr (sizeof(T) == 4) {
#pragma unroll
              for (int t = 0; t < 4; ++t)
                acc[qg][grp] = __builtin_amdgcn_mfma_f32_16x16x4f32(xf[grp][t], qf[qg][t],
                                                                    acc[qg][grp], 0, 0, 0);
            } else {
              acc[qg][grp] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  __builtin_bit_cast(bf16x8, xf[grp]), __builtin_bit_cast(bf16x8, qf[qg]),
                  acc[qg][grp], 0, 0, 0);
            }
          }
        }
      }
      // retire slice sl+1: the slices issued after it stay in flight
      const int younger = min(sl + NB - 1, nslice - 1) - (sl + 1);
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }

    // Epilogue: keys, 8-bit candidate mask per query group, park + insert.
    const int r = tb + 32 * w;
#pragma unroll
    for (int qg = 0; qg < NQG; ++qg) {
      const float tk = lk[qg][KP - 1];
      const int ti = li[qg][KP - 1];
      const bool qvalid = qcol[qg] < nq;
      uint32_t m = 0;
#pragma unroll
      for (int grp = 0; grp < 2; ++grp) {
        const int rowb = r + 16 * grp + 4 * g;
        f32x4v xa = {0.f, 0.f, 0.f, 0.f};
        if constexpr (MODE == MODE_L2) xa = *(const f32x4v*)(xaux + rowb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v = acc[qg][grp][i];
          const float key = MODE == MODE_L2 ? l2_from_ip(qa[qg], xa[i], v) : -v;
          acc[qg][grp][i] = key;
          const bool cand = qvalid && (rowb + i) < ntotal && lex_less(key, rowb + i, tk, ti);
          m |= (uint32_t)cand << (grp * 4 + i);
        }
      }
      if (m) {
#pragma unroll
        for (int grp = 0; grp < 2; ++grp)
#pragma unroll
          for (int i = 0; i < 4; ++i) spark[(grp * 4 + i) * 256 + tid] = acc[qg][grp][i];
        do {
          const int bi = __builtin_ctz(m);
          m &= m - 1;
          const int row = r + 16 * (bi >> 2) + 4 * g + (bi & 3);
          list_insert<KP, int>(lk[qg], li[qg], spark[bi * 256 + tid], row);
        } while (m);
      }
    }
    __syncthreads();  // the next tile's first slices overwrite the parking area
  }

  // Fold the 16 lists of each query (4 lane groups x 4 waves) in LDS, one
  // query group at a time; thread t < 16 folds query t with a 4-round tree.
  const int slot = w * 4 + g;  // 0..15
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) {
    __syncthreads();  // previous use of the LDS (parking or the last fold) is done
    const int base = (c16 * 16 + slot) * KP;
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      mk[base + j] = lk[qg][j];
      mi[base + j] = li[qg][j];
    }
    __syncthreads();
    for (int step = 1; step < 16; step <<= 1) {
      const int q = tid >> 4, s = tid & 15;
      if (q < 16 && (s & (2 * step - 1)) == 0) {
        float ok[KP];
        int oi[KP];
        const int a = (q * 16 + s) * KP, b = (q * 16 + s + step) * KP;
        merge2_sorted<KP, int>(mk + a, mi + a, mk + b, mi + b, ok, oi);
#pragma unroll
        for (int j = 0; j < KP; ++j) {
          mk[a + j] = ok[j];
          mi[a + j] = oi[j];
        }
      }
      __syncthreads();
    }
    const int qglob = qg * 16 + tid;
    if (tid < 16 && qglob < nq) {
      const int a = tid * 16 * KP;
      float* ok = pkey + ((int64_t)qglob * gridDim.x + blockIdx.x) * KP;
      int* oi = pid + ((int64_t)qglob * gridDim.x + blockIdx.x) * KP;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        ok[j] = mk[a + j];
        oi[j] = mi[a + j];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// skinny_plane_topk: the filter engine's deep bf16 stage for a FEW gathered
// queries (at most kPlaneQ, a device-side count), HBM-bound.  The x1 pass
// would multiply every database tile by a whole 256-query tile for them (a
// 10M-row pass of ~18 ms for 26 queries at C3 k = 60, profiles/r05t); this
// kernel streams the same bf16 plane once (30.7 GB at 10M x 1536: ~5 ms) and
// leaves the x1 pass's lane-list layout, so the stage's verification is
// unchanged.
//   Plane: tile-major (vs_internal.h plane_offset): tile t's 64-B step s of
//   its 256 rows is one 16-KB block.  Queries: the first kPlaneQ rows of the
//   gathered query plane's tile 0, same layout.  Block b of the grid (P =
//   gridDim.x blocks: the x1 deep stage's 4 * nsplit lane lists) takes tiles
//   [b * ntiles / P, (b + 1) * ntiles / P) and writes, per query, its top KL
//   (key -sum, row) to list b — every row of its tiles outside the list has a
//   key >= the list's last entry, the lane lists' contract.
//   Four waves; wave w owns rows 64 w .. 64 w + 63 of each tile (4 groups of
//   16) against the 64 queries (4 groups of 16): 16 v_mfma_f32_16x16x32_bf16
//   per 64-B step.  LDS-DMA into a ring of kPlaneNB images of 20 KB (16 KB of
//   rows, 4 KB of queries), chunk c of row r at c ^ ((r >> 2) & 3).
constexpr int kPlaneQ = 64;
constexpr int kPlaneNB = 4;
constexpr int kPlaneImg = 16384 + 4096;

template <int KL, int EL, int NQG, bool NT>
__global__ __launch_bounds__(256, 2) void skinny_plane_topk(
    const char* __restrict__ XH, const char* __restrict__ QH, int nksteps, int ntiles, int ntotal,
    const int* __restrict__ qcount, float* __restrict__ pkey, int* __restrict__ pid, int KP,
    const float* __restrict__ qs, const float* __restrict__ xs) {
  // NQG query groups of 16 (1: at most 16 queries, a quarter of the MFMAs and
  // fragment reads; 4: at most 64)
  // EL: the plane (FILTER_BF16: v_mfma_f32_16x16x32_bf16, key -sum; FILTER_I8:
  // v_mfma_i32_16x16x64_i8, key -(sum * (s_q * s_x)) — the x1 pass's keys)
  using Acc = typename std::conditional<EL == FILTER_I8, i32x4, f32x4>::type;
  const int cnt = *qcount;
  // uniform: the x1 deep pass (more than kPlaneQ) or the other variant takes it
  if (cnt <= 0 || cnt > 16 * NQG || (NQG > 1 && cnt <= 16)) return;
  constexpr int kFold = kPlaneQ * 16 * KL;  // [query][16 lane lists][KL]
  constexpr int kWords0 = kPlaneNB * kPlaneImg / 4;
  constexpr int kWords = kWords0 > 2 * kFold ? kWords0 : 2 * kFold;
  static_assert(2 * kWords * 4 <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(16))) float lds[kWords];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4;
  const int c16 = lane & 15;
  const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(lds);
  const int P = gridDim.x;
  const int t0 = (int)((int64_t)blockIdx.x * ntiles / P);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * ntiles / P);
  const int nst = (t1 - t0) * nksteps;  // steps of this block

  float lk[NQG][KL];
  int li[NQG][KL];
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) list_init<KL, int>(lk[qg], li[qg]);

  // DMA: lane L of a 1-KB piece moves 16 B of row (L >> 2) of a 16-row group,
  // chunk slot L & 3, reading chunk (L & 3) ^ ((row >> 2) & 3) (the swizzle)
  const uint32_t soff = (uint32_t)(lane >> 2) * 64u + (uint32_t)((lane & 3) ^ (lane >> 4)) * 16u;
  // this wave's pieces of a step: row pieces 4 w .. 4 w + 3, query piece w
  auto stage = [&](int gs) {
    const int t = t0 + gs / nksteps, st = gs - (gs / nksteps) * nksteps;
    const uint32_t base = lds0 + (uint32_t)((gs % kPlaneNB) * kPlaneImg);
    const char* xb = XH + ((int64_t)t * nksteps + st) * 16384;
    const char* qb = QH + (int64_t)st * 16384;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      skinny_glds_p<NT>(xb + (4 * w + i) * 1024, soff,
                        __builtin_amdgcn_readfirstlane(base + (uint32_t)(4 * w + i) * 1024u));
    // query piece w (NQG = 1: every wave the same piece 0, identical bytes to
    // identical LDS addresses, so every wave issues 5 loads per step)
    const int qp = NQG == 1 ? 0 : w;
    skinny_glds(qb + qp * 1024, soff,
                __builtin_amdgcn_readfirstlane(base + 16384u + (uint32_t)qp * 1024u));
  };
  // fragment reads: row r (of the 16 KB rows, or of the queries), chunk g
  auto frag = [&](const char* img, int r) -> i32x4 {
    return *(const i32x4*)(img + r * 64 + ((g ^ ((r >> 2) & 3)) * 16));
  };
  float qsc[NQG];
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) qsc[qg] = EL == FILTER_I8 ? qs[16 * qg + c16] : 0.0f;

  if (nst > 0) {
#pragma unroll
    for (int i = 0; i < kPlaneNB - 1; ++i)
      if (i < nst) stage(i);  // uniform
    if (nst >= 3) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (nst >= 2) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    Acc acc[4][NQG];
    for (int gs = 0; gs < nst; ++gs) {
      const int st = gs % nksteps;
      if (st == 0) {
#pragma unroll
        for (int rg = 0; rg < 4; ++rg)
#pragma unroll
          for (int qg = 0; qg < NQG; ++qg) acc[rg][qg] = Acc{};
      }
      // step gs+NB-1 into the image step gs-1 used (every wave passed the
      // barrier after reading it)
      if (gs + kPlaneNB - 1 < nst) stage(gs + kPlaneNB - 1);
      const char* img = (const char*)lds + (gs % kPlaneNB) * kPlaneImg;
      i32x4 a[4], b[NQG];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag(img, 64 * w + 16 * i + c16);
#pragma unroll
      for (int i = 0; i < NQG; ++i) b[i] = frag(img + 16384, 16 * i + c16);
#pragma unroll
      for (int rg = 0; rg < 4; ++rg)
#pragma unroll
        for (int qg = 0; qg < NQG; ++qg) {
          if constexpr (EL == FILTER_I8)
            acc[rg][qg] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[rg], b[qg], acc[rg][qg], 0, 0, 0);
          else
            acc[rg][qg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                __builtin_bit_cast(bf16x8, a[rg]), __builtin_bit_cast(bf16x8, b[qg]), acc[rg][qg],
                0, 0, 0);
        }
      if (st == nksteps - 1) {
        // tile done: lane holds rows 16 rg + 4 g + i of the wave's 64 for
        // query 16 qg + c16; keys -sum, rows past the corpus never enter
        const int row0 = (t0 + gs / nksteps) * 256 + 64 * w + 4 * g;
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          f32x4 fx = {0.f, 0.f, 0.f, 0.f};
          if constexpr (EL == FILTER_I8) fx = *(const f32x4*)(xs + row0 + 16 * rg);
#pragma unroll
          for (int qg = 0; qg < NQG; ++qg)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int row = row0 + 16 * rg + i;
              float key;
              if constexpr (EL == FILTER_I8)
                key = -((float)acc[rg][qg][i] * (qsc[qg] * fx[i]));  // x1_key<FILTER_I8>
              else
                key = -acc[rg][qg][i];
              if (row < ntotal && lex_less(key, row, lk[qg][KL - 1], li[qg][KL - 1]))
                list_insert<KL, int>(lk[qg], li[qg], key, row);
            }
        }
      }
      // retire step gs+1: the steps issued after it stay in flight
      const int younger = min(gs + kPlaneNB - 1, nst - 1) - (gs + 1);
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }

  // fold: query q's 16 lists (4 waves x 4 lane groups) in LDS, tree merge,
  // list b of every query slot written (slots past the count are never read)
  float* mk = lds;
  int* mi = (int*)(lds + kFold);
  __syncthreads();
  const int slot = w * 4 + g;
#pragma unroll
  for (int qg = 0; qg < NQG; ++qg) {
    const int base = ((16 * qg + c16) * 16 + slot) * KL;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      mk[base + j] = lk[qg][j];
      mi[base + j] = li[qg][j];
    }
  }
  __syncthreads();
  for (int step = 1; step < 16; step <<= 1) {
    // 64 queries x 8 pairs at step 1: 512 merges over 256 threads, two each
    for (int m = tid; m < 16 * NQG * 16; m += 256) {
      const int q = m >> 4, sl = m & 15;
      if ((sl & (2 * step - 1)) != 0) continue;
      float ok[KL];
      int oi[KL];
      const int a0 = (q * 16 + sl) * KL, b0 = (q * 16 + sl + step) * KL;
      merge2_sorted<KL, int>(mk + a0, mi + a0, mk + b0, mi + b0, ok, oi);
#pragma unroll
      for (int j = 0; j < KL; ++j) {
        mk[a0 + j] = ok[j];
        mi[a0 + j] = oi[j];
      }
    }
    __syncthreads();
  }
  for (int m = tid; m < 16 * NQG * KL; m += 256) {
    const int q = m / KL, j = m - q * KL;
    const int64_t o = ((int64_t)q * P + blockIdx.x) * KP + j;
    pkey[o] = mk[q * 16 * KL + j];
    pid[o] = mi[q * 16 * KL + j];
  }
}

// The plane passes' row pieces with the non-temporal policy (default; env
// VS_SKINNY_NT=0 keeps the default policy, for A/B; read at every search)
static bool skinny_nt() {
  const char* e = getenv("VS_SKINNY_NT");
  return !e || atoi(e) != 0;
}

hipError_t launch_skinny_plane(int filter, const void* XH, const void* QH, int64_t ld, int ntotal,
                               const int* qcount, const float* qs, const float* xs, Partials part,
                               hipStream_t st, int nq_hint) {
  const int64_t ldb = ld * (filter == FILTER_I8 ? 1 : 2);
  if (ldb % 64 != 0 || part.KP < 8 || part.P < 1 || !qcount ||
      (filter == FILTER_I8 && (!qs || !xs)))
    return hipErrorInvalidValue;
  const int nksteps = (int)(ldb / 64);
  const int ntiles = (ntotal + 255) / 256;
  // nq_hint: the host's bound on the count (0: unknown, up to kPlaneQ): the
  // 16-query variant runs for counts <= 16, the 64-query one above; each exits
  // on the other's counts, so both are launched unless the bound decides
  const bool nt = skinny_nt();
#define VS_SP(EL_, NQG_)                                                                          \
  do {                                                                                            \
    if (nt)                                                                                       \
      hipLaunchKernelGGL((skinny_plane_topk<8, EL_, NQG_, true>), dim3(part.P), dim3(256), 0, st, \
                         (const char*)XH, (const char*)QH, nksteps, ntiles, ntotal, qcount,       \
                         part.key, part.id, part.KP, qs, xs);                                    \
    else                                                                                          \
      hipLaunchKernelGGL((skinny_plane_topk<8, EL_, NQG_, false>), dim3(part.P), dim3(256), 0,   \
                         st, (const char*)XH, (const char*)QH, nksteps, ntiles, ntotal, qcount,   \
                         part.key, part.id, part.KP, qs, xs);                                    \
  } while (0)
  if (filter == FILTER_I8) {
    VS_SP(FILTER_I8, 1);
    if (nq_hint <= 0 || nq_hint > 16) VS_SP(FILTER_I8, 4);
  } else {
    VS_SP(FILTER_BF16, 1);
    if (nq_hint <= 0 || nq_hint > 16) VS_SP(FILTER_BF16, 4);
  }
#undef VS_SP
  return hipGetLastError();
}
int skinny_plane_max_queries() { return kPlaneQ; }

template <int KP, int MODE, typename T>
static hipError_t skinny_launch_t(int nq, const T* X, const float* xaux, const T* Q,
                                  const float* qaux, int64_t ld, int ntotal, int nblocks,
                                  Partials part, hipStream_t st, const int* qcount) {
  const int nt256 = (ntotal + 255) & ~255;
  int rpb = (nt256 + nblocks - 1) / nblocks;
  rpb = (rpb + 255) & ~255;  // whole 256-row tiles
  if (nq <= 16)
    hipLaunchKernelGGL((skinny_topk<KP, MODE, T, 1>), dim3(nblocks), dim3(256), 0, st, X, xaux,
                       Q, qaux, ld, nq, ntotal, rpb, part.key, part.id, qcount);
  else
    hipLaunchKernelGGL((skinny_topk<KP, MODE, T, 2>), dim3(nblocks), dim3(256), 0, st, X, xaux,
                       Q, qaux, ld, nq, ntotal, rpb, part.key, part.id, qcount);
  return hipGetLastError();
}

template <int KP>
static hipError_t skinny_launch_kp(int mode, int nq, const void* X, int esize, const float* xaux,
                                   const void* Q, const float* qaux, int64_t ld, int ntotal,
                                   int nblocks, Partials part, hipStream_t st, const int* qcount) {
  if (esize == 4) {
    if (mode == MODE_L2)
      return skinny_launch_t<KP, MODE_L2, float>(nq, (const float*)X, xaux, (const float*)Q, qaux,
                                                 ld, ntotal, nblocks, part, st, qcount);
    return skinny_launch_t<KP, MODE_IP, float>(nq, (const float*)X, xaux, (const float*)Q, qaux,
                                               ld, ntotal, nblocks, part, st, qcount);
  }
  if (mode == MODE_L2)
    return skinny_launch_t<KP, MODE_L2, uint16_t>(nq, (const uint16_t*)X, xaux,
                                                  (const uint16_t*)Q, qaux, ld, ntotal, nblocks,
                                                  part, st, qcount);
  return skinny_launch_t<KP, MODE_IP, uint16_t>(nq, (const uint16_t*)X, xaux, (const uint16_t*)Q,
                                                qaux, ld, ntotal, nblocks, part, st, qcount);
}

hipError_t launch_skinny_topk(int KP, int mode, int nq, const void* X, int esize,
                              const float* xaux, const void* Q, const float* qaux, int64_t ld,
                              int ntotal, int nblocks, Partials part, hipStream_t st,
                              const int* qcount) {
  if (nq < 1 || nq > kSkinnyMaxQ || part.KP != KP || part.P != nblocks ||
      (ld * esize) % 128 != 0 || (esize != 4 && esize != 2) || (mode != MODE_IP && mode != MODE_L2))
    return hipErrorInvalidValue;
  switch (KP) {
    case 8:
      return skinny_launch_kp<8>(mode, nq, X, esize, xaux, Q, qaux, ld, ntotal, nblocks, part, st,
                                 qcount);
    case 16:
      return skinny_launch_kp<16>(mode, nq, X, esize, xaux, Q, qaux, ld, ntotal, nblocks, part,
                                  st, qcount);
    case 32:
      return skinny_launch_kp<32>(mode, nq, X, esize, xaux, Q, qaux, ld, ntotal, nblocks, part,
                                  st, qcount);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace vs
