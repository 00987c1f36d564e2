// vs_gemm_x1.hip — the filter pass of the filter-and-verify engine: one
// low-precision MFMA product per fp32 product, fused with per-lane candidate
// lists.
//
// Every fp32 index keeps, beside its fp32 rows, a "filter plane" copy of every
// row ([capacity][ld], row-major) and the squared norm of each row's residual
// x - plane(x).  Two planes exist (vs_internal.h, Filter):
//   int8 (default): code = rint(x / s) with one scale s = max|x| / 127 per row;
//     the kernel multiplies codes on v_mfma_i32_32x32x32_i8 (exact int32 sums,
//     twice the bf16 MFMA rate, 64 elements per 64-B step) and scales the sum
//     by s_q * s_x in the epilogue;
//   bf16: round-to-nearest-even copies on v_mfma_f32_32x32x16_bf16.
// A search converts its queries the same way and the kernel below scores every
// (query, row) pair with the one product plane(q) . plane(x) — a plain GEMM over
// Q (nq x d) and X (N x d) whose output never leaves the chip: each lane keeps
// the best approximate keys of its queries.  The exact answer is then proved and
// produced by verify_rescore_kernel (below): the candidates are rescored in
// fp64 from the fp32 rows, and a rigorous bound on |approx - exact| decides
// whether the candidate set must contain the exact top-M.
//
// Tile: 256 database rows x 256 queries per workgroup of 8 waves (two per SIMD,
// one workgroup per CU).  Wave w owns rows [128 (w&1), +128) and queries
// [64 (w>>1), +64): 4 x 2 accumulators of 32x32 (128 registers); lane l sees
// queries c = l&31 of its two 32-query blocks and keeps one sorted list of KR
// entries per query (lanes l and l+32 hold disjoint rows of the same query).
// K advances 64 B per row per step (32 bf16 / 64 int8 elements) through a ring of NBUF LDS
// images (both operand tiles of one step, 32 KB), filled by
// global_load_lds_dwordx4 (LDS-DMA) NBUF-1 steps ahead; see gemm_topk_x1
// below for the step schedule.
//
// Two kinds of launch (template flag DUMP), per search:
//  * list launches (the first launch of a pass, gathered batches, the bf16
//    L2 / cosine kernels): the epilogue of every 256-row tile reduces each
//    lane's 16 keys of a 32-row block to their maximum and, only when the
//    block can enter the lane's list, inserts its rows one by one;
//  * dump launches (every later launch of an int8 or bf16 inner-product
//    pass): the lists stay in memory; the epilogue compares each block with
//    its list's floor (the query's CUT, x1_qcut, set from the first launch's
//    lists, or the list's own last entry) and, for the rare block that may
//    hold a row below it, stores one (row, raw sum) pair per row that clears
//    the per-row threshold to the list's next dump slot; x1_replay (between
//    segments of launches) admits the dumped rows into the lists exactly as a
//    list launch would have — same keys, same order, same admission rule — so
//    both kinds leave the same lists.
// The lists are per lane, so a list launch pays for a wave's rows whenever ANY
// of its 64 lanes admits one (an exec-masked insertion chain per block that
// passes somewhere): about a sixth of the int8 pass (profiles/r04a/x1_probes.txt:
// 3.45 ms per dispatch with the candidate work, 2.86 ms with the epilogue's
// per-block test alone).  A dump costs one 8-B store per candidate row on the
// lanes that pass.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "vs_device.h"

// Diagnostic builds only (tools/x1_probe.sh; wrong results by design): a mask
// of ablations — 1 no LDS-DMA, 2 no fragment reads, 4 no mid-step barrier,
// 8 no epilogue, 16 no database pieces, 32 no query pieces, 64 no vmcnt wait in
// the loop, 128 the epilogue's per-block test alone (no block ever passes).
#ifndef VS_X1_PROBE
#define VS_X1_PROBE 0
#endif
#define VS_X1_P(bit) ((VS_X1_PROBE & (bit)) != 0)

namespace vs {

// Diagnostic builds only (VS_X1_STAMP=1, tools/build_variant.sh): per-segment
// s_memtime sums of the step schedules, [group (waves 0-3 | 4-7)][segment]
// (segments: load issue, vmcnt wait, barrier 1, matrix issue, barrier 2,
// epilogue), added once per wave at the end; read by vs_x1_stamps.  The real
// kernel has no stamp.
#ifndef VS_X1_STAMP
#define VS_X1_STAMP 0
#endif
constexpr int kStampSeg = 9;  // + inside the epilogue: reject, factor loads, keys/inserts
constexpr int kStampCnt = 3;  // epilogue counts: factor loads, blocks inserting, inserts
constexpr int kStampN = 2 * (kStampSeg + kStampCnt) + 2;
__device__ unsigned long long g_x1_stamps[kStampN];

namespace {

constexpr int kT = 256;               // rows (and queries) per tile
constexpr int kNbuf = 5;              // LDS images in the ring (4: -1 %, profiles/r02y)
constexpr int kX1ChunkTiles = 64;     // database tiles per workgroup per launch
// dump slots (candidate rows) per lane list and segment: a segment of
// doubling data meets ~8 rows below a list's floor, a hybrid launch's dump part
// (three times its list part) ~24, with a tail: the dump part beats the list
// part's 8th row at least n times when at most 7 of the best 8 + n rows lie in
// the list part, Binomial(8 + n, 1/4) <= 7: ~2e-4 per list at n = 64 (a fifth of
// C2's queries, with 512 lists each, handed on), ~1e-8 at n = 128
constexpr int kDumpMaxR = 128;
// The step schedule of a launch: 1 = fragment reads half a step ahead, DMA
// pieces between the MFMAs; 2 = separate load and matrix segments.  Measured
// per plane and launch kind (A/B builds: VS_X1_SCHED_I8 forces one for every
// int8 launch): int8 list launches are faster on 1 (C2 390k vs 337k
// queries/s, C4 465k vs 437k students/s), int8 dump launches on 2 (C3 70.8k
// vs 68.9k; profiles/r04a/r04e_sched_dump_ab.txt), bf16 on 2 (clustered
// 34.4k vs 32.5k, profiles/r03_ab_sched.txt).
#ifndef VS_X1_SCHED_I8
#define VS_X1_SCHED_I8 0
#endif
// A/B builds only (tools/build_variant.sh -DVS_X1_SEGDMA=1): the segmented
// schedule's four LDS-DMA pieces of step s+3 issued between the MFMAs of the
// matrix segment (one per four MFMAs) instead of in the load segment.
#ifndef VS_X1_SEGDMA
#define VS_X1_SEGDMA 0
#endif
// A hybrid launch (mostly dump tiles) takes the dump launches' schedule.
constexpr int x1_sched(int el, bool dump, bool hyb = false) {
  return el != FILTER_I8 ? 2 : VS_X1_SCHED_I8 ? VS_X1_SCHED_I8 : dump || hyb ? 2 : 1;
}
// The passes with a dump form: inner product on either plane (every key
// follows from the raw sum and, for int8, the row factor the replay reads).
// Not the cosine: its bound is relative (B ~ 2 rho, ~0.02 at d = 1536 for
// int8), wide beside the similarity spread of high-dimensional rows, so only
// the lists' own floors hold its dumps down, and its row factors (s_x / |x|)
// spread widely, so a launch-wide factor bound passes ~70 rows per list and
// segment (a d = 128 self-join of Gaussian rows: 3M lists past their slots).
// A form with the list launches' per-group bounds and exact keys before the
// dump (built, exact) made C4 slower: 439k vs 467k students/s at 4-5
// launches per pass (profiles/r04w/ab_c4_cosine_dump.txt).  The bf16 L2 /
// cosine keys also need the row norms in the kernel.
constexpr bool x1_has_dump(int mode, int el) {
  return mode == MODE_IP || (mode == MODE_COS && el == FILTER_I8);
}
// The int8 cosine's dump form (its folded factors s_x / |x| take the place of
// s_x; key and bound as in its list launches) is used only with VS_X1_COSDUMP=1
// (A/B; read at every search): its cut lies behind the lists' own floors, so
// it stores about as many rows as list launches insert (C4 440-469k vs 471k
// students/s, profiles/r05o).
static bool x1_cos_dump_on() {
  const char* e = getenv("VS_X1_COSDUMP");
  return e && atoi(e) != 0;
}

__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// Four elements of a stored row as floats: fp32 rows, or bf16 rows widened
// (exactly) — the verification of a bf16 index's int8 plane rescores the
// stored bf16 values.
__device__ __forceinline__ f32x4 row4(const float* __restrict__ p) { return *(const f32x4*)p; }
__device__ __forceinline__ f32x4 row4(const uint16_t* __restrict__ p) {
  const uint2 u = *(const uint2*)p;
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u),
               __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xFFFF0000u)};
}

__device__ __forceinline__ bf16x8 as_bf(const uint4& u) { return __builtin_bit_cast(bf16x8, u); }
__device__ __forceinline__ i32x4 as_i4(const uint4& u) { return __builtin_bit_cast(i32x4, u); }

// One 32x32 block of one 64-B sub-step: C (+)= A . B on the plane's MFMA.
template <int EL>
using AccT = typename std::conditional<EL == FILTER_I8, i32x16, f32x16>::type;
template <int EL>
__device__ __forceinline__ AccT<EL> mfma_blk(const uint4& a, const uint4& b, const AccT<EL>& c) {
  if constexpr (EL == FILTER_I8)
    return __builtin_amdgcn_mfma_i32_32x32x32_i8(as_i4(a), as_i4(b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(as_bf(a), as_bf(b), c, 0, 0, 0);
}

// LDS-DMA of 16 B per lane into the wave-uniform LDS byte address `lds` (M0 is
// written and restored inside the statement; cdna_hip_programming.md §5.7).
// hipcc does not count it, so it inserts no waits of its own around it: the
// caller retires it with a counted vmcnt before the barrier that precedes the
// ds_reads of that image (the builtin form makes hipcc assume every later LDS
// read may alias it and drain vmcnt to 0 before them).  No VGPR destination,
// so no register hazard.
// The source is a uniform base (SGPR pair) plus a 32-bit per-lane offset: no
// 64-bit address VGPRs beside the accumulators.
__device__ __forceinline__ void glds16(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}

// Row order inside database tile t: LDS slot s holds tile row s ^ tile_perm(t)
// (bits 2..7, so 4-row groups stay contiguous).  The slot decides which lane
// list sees a row; without the permutation a row's list would depend only on
// row % 256, and data laid out periodically (rows of one cluster every 1024
// rows, say) would crowd a quarter of a query's lists, pulling the wide
// check's floor T toward the top and failing its bound.
__device__ __forceinline__ int tile_perm(int t) {
  return (int)(((uint32_t)t * 2654435761u) >> 24) & 0xFC;
}

__device__ __forceinline__ int sel16i(const i32x16& v, int i) {
  int r = v[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) r = i == j ? v[j] : r;
  return r;
}

__device__ __forceinline__ float sel4x4(const f32x4 (&v)[4], int i) {
  float r = v[0][0];
#pragma unroll
  for (int j = 1; j < 16; ++j) r = i == j ? v[j >> 2][j & 3] : r;
  return r;
}

// int8 candidate threshold: an integer T with fl(fl(float(a)) * c) <= lim for
// every int32 a <= T (c > 0; the scaled score is monotone in a), from an
// approximate quotient minus a margin, then checked: INT_MIN (every row a
// candidate) when the check fails.  A smaller T only admits more candidates.
__device__ __forceinline__ int i8_threshold(float lim, float c) {
  const float q = lim * __builtin_amdgcn_rcpf(c);
  const float qm = q > 0.0f ? q * (1.0f - 0x1p-20f) : q * (1.0f + 0x1p-20f);
  float fl = floorf(qm) - 2.0f;
  fl = fminf(fmaxf(fl, -2147483520.0f), 2147483520.0f);  // in int range (NaN -> lower bound)
  const int T = (int)fl;
  return (float)T * c <= lim ? T : INT_MIN;
}

__device__ __forceinline__ float sel16(const f32x16& v, int i) {
  float r = v[0];
#pragma unroll
  for (int j = 1; j < 16; ++j) r = i == j ? v[j] : r;
  return r;
}

// The approximate key of a row from its raw sum (int8: the exact int32 sum
// times the two factors, three fp32 roundings, five with the cosine's folded
// inverse norms — xs holds s_x (IP) or s_x / |x| (COS), qsc s_q or s_q / |q|;
// bf16 inner product: -sum exactly).  One expression for the list epilogue and
// the replay, so both produce the same bits.
template <int EL>
__device__ __forceinline__ float x1_key(int sum_bits, float qsc, float fx) {
  if constexpr (EL == FILTER_I8) return -((float)sum_bits * (qsc * fx));
  else return -__int_as_float(sum_bits);
}

}  // namespace

// ---------------------------------------------------------------------------
// The step schedule.  Each 32-element step is two sub-steps of 16 (8 MFMAs per
// wave each), cut at its middle by the one barrier of the step, and the
// fragment reads run one half-step ahead of the MFMAs:
//     MFMAs of sub-step 0 (fragments read during the previous step)
//     ds_read the sub-step 1 fragments
//     wait for this wave's pieces of step s+1, s_barrier
//     LDS-DMA of step s+NBUF-1 into the image step s-1 used (every wave has
//       passed this barrier, so every read of that image is done)
//     MFMAs of sub-step 1, then ds_read sub-step 0 of step s+1 (its image is
//       complete: every wave's pieces were retired before this barrier)
// so the LDS read latency after a barrier hides under MFMAs instead of
// stalling both waves of a SIMD at every step.  The LDS-DMA steps are retired
// with a COUNTED vmcnt (the younger NBUF-2 steps stay in flight across the raw
// s_barrier; cdna_hip_programming.md "Pipelining across barriers"); loads past
// the last step re-read it (unconditional loads keep the count fixed).  64-B
// LDS rows: chunk c of row r at c ^ ((r >> 2) & 3) — conflict-free ds_read_b128
// for the 32x32x16 fragments, and one per-lane source offset for every 16-row
// group.  The first sub-step of every tile multiplies into a zero accumulator
// (the MFMA's inline-constant C), so no register clearing between tiles.  Load
// and position cursors are incremental (no divisions in the loop).
// A dump launch's stores (rare: a block below the cut) are vector-memory
// operations younger than the DMA pieces in flight: a counted wait after them
// retires more than its step needs (over-waits), never less.
//
// XCD blocking (grids of 8 S workgroups; workgroup b runs on XCD b % 8, in slot
// order b / 8 there): the S workgroups of an XCD take QG query tiles x DG
// database splits (QG = min(nqt, qg)), so each XCD's L2 holds QG query tiles'
// slices (QG x 16 KB per step) and serves a database tile to QG workgroups;
// slot / QG orders the splits, so with two rounds of workgroups per CU each
// round covers its own DG / 2 splits.  Other grids: a plain dealing.
template <int KR, int MODE, bool DUMP, int EL, bool HYB = false>
__global__ __launch_bounds__(512, 1) void gemm_topk_x1(
    const char* __restrict__ XH, const float* __restrict__ xs, const float* __restrict__ xaux,
    const char* __restrict__ QH, const float* __restrict__ qs, const float* __restrict__ qaux,
    int nqa, int nksteps, int ntotal, int ntiles, int nsplit, int nqt, int qtile0, int64_t self0,
    const int* __restrict__ qrow, const int* __restrict__ qcount, int chunk, int chunk_end,
    int nchunk, int KP, int qg, float* __restrict__ pkey, int* __restrict__ pid,
    const float* __restrict__ xgmax, const float* __restrict__ xgmin, const float* __restrict__ qcut,
    int* __restrict__ dcount, int* __restrict__ dslot, int dR, int qskip) {
  static_assert(!DUMP || x1_has_dump(MODE, EL), "dump form");
  static_assert(!HYB || (!DUMP && x1_has_dump(MODE, EL)), "hybrid launch");
  constexpr int NBUF = kNbuf;
  constexpr int kStepB = kT * 64;  // one operand tile of one 32-element step: 16 KB
  constexpr int D = NBUF - 1;      // steps in flight
  static_assert(NBUF * 2 * kStepB <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[NBUF * 2 * kStepB];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5;
  const int c32 = lane & 31;
  const int wr = w & 1;
  const int wq = w >> 1;

  int qt, sp;
  {
    const int nblk = gridDim.x;
    const int b = blockIdx.x;
    const int qga = qg < 0 ? -qg : qg;  // qg < 0: no rounds of groups (A/B)
    const int QG = nqt < qga ? nqt : qga;
    const int G = nqt / QG;
    const int S = nblk >> 3;
    if ((nblk & 7) == 0 && nqt * nsplit == nblk && nqt % QG == 0 && G <= 8 && 8 % G == 0 &&
        S % QG == 0) {
      const int xcd = b & 7, slot = b >> 3, DG = S / QG;
      qt = (xcd % G) * QG + slot % QG;
      sp = (xcd / G) * DG + slot / QG;
    } else if (qg > 0 && (nblk & 7) == 0 && nqt * nsplit == nblk && nqt % QG == 0 && G % 8 == 0) {
      // more query-tile groups than XCDs (C4's 65,536-student chunks: 256 query
      // tiles): XCD x takes groups x, x + 8, ... one after another, each as QG
      // query tiles x every split in slot order, so the workgroups an XCD runs
      // together share their database tiles and their QG query tiles in its L2
      // (a plain dealing put 32 different query tiles on an XCD at once)
      const int xcd = b & 7, slot = b >> 3, per = QG * nsplit;
      const int gi = slot / per, rem = slot - gi * per;
      qt = (gi * 8 + xcd) * QG + rem % QG;
      sp = rem / QG;
    } else {
      const int xcd = b & 7, slot = b >> 3, qq = nblk >> 3, rr = nblk & 7;
      const int lb = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + slot;
      qt = lb % nqt;
      sp = lb / nqt;
    }
  }
  // a gathered batch (device-side count): query tiles past it have nothing to do
  // (qskip: a gathered stage of at most qskip queries is skinny_plane_topk's)
  if (qcount && (qt * kT >= *qcount || *qcount <= qskip)) return;  // uniform
  const int s0 = (int)((int64_t)sp * ntiles / nsplit);
  const int s1 = (int)((int64_t)(sp + 1) * ntiles / nsplit);
  const int t0 = s0 + (int)((int64_t)(s1 - s0) * chunk / nchunk);
  // parts [chunk, chunk_end) of the split's nchunk (a launch usually covers one)
  const int t1 = s0 + (int)((int64_t)(s1 - s0) * chunk_end / nchunk);
  // Hybrid launch: the first quarter of the workgroup's tiles as a list
  // launch, the rest as a dump launch whose floor is each list's own last
  // entry after that quarter (a top-8 list over n rows is beaten by ~8 of every
  // next n: ~24 dumps per list, within the slots)
  const int tsw = HYB ? t0 + (t1 - t0 + 3) / 4 : t1;

  int gq[2], selfrow[2];
  float qa[2], qsc[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    gq[qb] = qt * kT + 64 * wq + 32 * qb + c32;
    qa[qb] = 0.0f;
    if constexpr (MODE == MODE_L2 || (MODE == MODE_COS && EL != FILTER_I8))
      qa[qb] = gq[qb] < nqa ? qaux[gq[qb]] : 0.0f;
    qsc[qb] = 0.0f;
    if constexpr (EL == FILTER_I8) qsc[qb] = gq[qb] < nqa ? qs[gq[qb]] : 0.0f;
    selfrow[qb] = qrow ? (gq[qb] < nqa ? qrow[gq[qb]] : -1) : self0 >= 0 ? (int)(self0 + gq[qb]) : -1;
  }
  const int P = nsplit * 4;
  const int pl = sp * 4 + wr * 2 + h;
  // List launches: the lane's sorted lists (admission limit: the last entry).
  // Dump launches: the query's cut (padding queries: nothing passes) and the
  // lane list's running dump count over the search's launches.
  // dump launches keep no list (the arrays are never touched there: no
  // registers); the epilogue's list branch is a template of its dump tag, so
  // it must type-check in every kernel
  constexpr int KL = KR;
  float lk[2][KL];
  int li[2][KL];
  float tq[2] = {0.0f, 0.0f};
  int dc[2] = {0, 0};
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    if constexpr (DUMP) {
      // the cut, or the list's own last entry after the first launch when
      // that is lower (a row at or above it can never enter this list: its
      // last entry only falls)
      const int64_t o = ((int64_t)gq[qb] * P + pl) * KP + KR - 1;
      float tl = qcut[gq[qb]];
      if (pid[o] >= 0) tl = fminf(tl, pkey[o]);
      tq[qb] = gq[qb] < nqa ? tl : -FLT_MAX;
      dc[qb] = dcount[(int64_t)gq[qb] * P + pl];
      asm volatile("" ::"v"(tq[qb]), "v"(dc[qb]));
    } else {
      const int64_t o = ((int64_t)gq[qb] * P + pl) * KP;
      if (chunk == 0) {
        list_init<KR, int>(lk[qb], li[qb]);
      } else {
#pragma unroll
        for (int e = 0; e < KR; ++e) {
          lk[qb][e] = pkey[o + e];
          li[qb][e] = pid[o + e];
        }
      }
#pragma unroll
      for (int e = 0; e < KR; ++e) asm volatile("" ::"v"(lk[qb][e]), "v"(li[qb][e]));
    }
    asm volatile("" ::"v"(qa[qb]));
    if constexpr (EL == FILTER_I8) asm volatile("" ::"v"(qsc[qb]));
  }

  if (t1 > t0) {  // uniform over the workgroup
    // Planes are tile-major (vs_internal.h plane_offset): the 64-B step s of
    // the 256 rows of tile t is one contiguous 16-KB block, so a DMA piece (16
    // rows x 64 B) reads 1 KB of consecutive bytes — eight whole 128-B lines,
    // not sixteen half lines of sixteen row-major rows.
    // per-lane DMA source: row (lane >> 2) of a 16-row piece, 16-B chunk
    // swizzled by the LDS slot (c ^ ((slot >> 2) & 3))
    const uint32_t soff = (uint32_t)(lane >> 2) * 64u + (uint32_t)((lane & 3) ^ (lane >> 4)) * 16u;
    const int fsw = (c32 >> 2) & 3;
    const char* qtile = QH + (int64_t)(qtile0 + qt) * nksteps * kStepB + (uint32_t)(32 * w) * 64u;
    const uint32_t lds0 = (uint32_t)(uintptr_t)VS_LDS(smem);
    const int nsteps = (t1 - t0) * nksteps;

    // load cursor: the step it issues next (past the end it keeps re-reading
    // the last step: unconditional loads keep the vmcnt counts fixed)
    int ls = 0, lt = t0, lk_ = 0, lbuf = 0;
    // the load tile's permuted source rows: slot 32 w + 16 p + (lane >> 2) of
    // piece p reads row (32 w + 16 p) ^ (f & 0xF0) + ((lane >> 2) ^ (f & 0x0C))
    // (the two parts occupy disjoint bits): one lane offset, a uniform rest
    uint32_t xlane = 0;
    int xhi = 0;
    auto set_xoff = [&](int tt) {  // once per tile; the lane id is re-derived
      const int f = tile_perm(tt);
      const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      xhi = f & 0xF0;
      xlane = (uint32_t)((ln >> 2) ^ (f & 0x0C)) * 64u + (uint32_t)((ln & 3) ^ (ln >> 4)) * 16u;
    };
    set_xoff(t0);
    // Segmented schedule: the load cursor's step as two running uniform
    // pointers (X: the lower of the wave's two permuted 16-row groups; Q: the
    // wave's query rows) and a lane offset per X group (both >= 0: the groups
    // differ in bit 4 of the row), so a step's four pieces cost two 64-bit
    // adds and one asm block (stage_step) instead of ~40 scalar instructions
    // of address arithmetic and M0 saves
    // (inner product only: the bf16 L2 / cosine list kernels have no registers
    // to spare for the two lane offsets)
    constexpr bool kSeg = x1_sched(EL, DUMP, HYB) == 2 && MODE == MODE_IP;
    const char* xstep = nullptr;
    const char* qstep = nullptr;
    uint32_t xl0 = 0, xl2 = 0;
    auto set_step_ptrs = [&]() {
      const int r0 = (32 * w) ^ xhi, r2 = (32 * w + 16) ^ xhi;
      xstep = XH + ((int64_t)lt * nksteps + lk_) * kStepB + (uint32_t)(r0 & ~16) * 64u;
      qstep = qtile + (int64_t)lk_ * kStepB;
      xl0 = xlane + (uint32_t)(r0 & 16) * 64u;
      xl2 = xlane + (uint32_t)(r2 & 16) * 64u;
    };
    if constexpr (kSeg) set_step_ptrs();

    // int8 dump launches: one integer threshold per list for the whole launch
    // (its floor is fixed, and the factor bound is the launch's: the maximum
    // of its tiles' group maxima), so the per-block test is a maximum and a
    // compare with no per-tile loads or threshold arithmetic
    // A floor above 0 (every row of the list so far scored below 0: queries
    // pointing away from the data) needs the SMALLEST factor instead: a row
    // with a negative sum scores highest with its smallest factor, so it can
    // clear the limit only if fl(sum * fl(s_q * fmin)) does (rows with sums
    // >= 0 always clear it, and the threshold is below 0).
    int Tq[2] = {0, 0};
    float fm = 0.0f, fn = FLT_MAX;  // the dump tiles' largest and smallest row factors
    auto set_Tq = [&]() {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float c = qsc[qb] * fm, cn = qsc[qb] * fn, last = tq[qb];
        Tq[qb] = (c > 0.0f && -last >= 0.0f)                    ? i8_threshold(-last, c)
                 : (cn > 0.0f && cn <= FLT_MAX && -last < 0.0f) ? min(i8_threshold(-last, cn), -1)
                 : (c > 0.0f || -0.0f < last)                   ? INT_MIN
                                                                : INT_MAX;
        asm volatile("" ::"v"(Tq[qb]));
      }
    };
    // the launch's (a hybrid launch: its dump part's) largest and smallest
    // row factor
    auto set_factor_bounds = [&](int ta) {
      const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
      for (int g = 16 * ta + ln; g < 16 * t1; g += 64) {
        fm = fmaxf(fm, xgmax[g]);
        fn = fminf(fn, xgmin[g]);
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        fm = fmaxf(fm, __shfl_xor(fm, m));
        fn = fminf(fn, __shfl_xor(fn, m));
      }
    };
    if constexpr (DUMP && EL == FILTER_I8) {
      set_factor_bounds(t0);
      set_Tq();
    }
    // Hybrid launch, at the end of its list part: the lists go to memory (the
    // replay after the launch admits the dumps into them), each list's floor
    // for the dump part is min(cut, its last entry)
    auto to_dump_mode = [&]() {
      if constexpr (HYB) {
        const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
        const int pl1 = sp * 4 + wr * 2 + (ln >> 5);
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const int64_t g = (int64_t)(qt * kT + 64 * wq + 32 * qb + (ln & 31)) * P + pl1;
          const int64_t o = g * KP;
#pragma unroll
          for (int e = 0; e < KR; ++e) {
            pkey[o + e] = lk[qb][e];
            pid[o + e] = li[qb][e];
          }
          for (int e = KR; e < KP; ++e) {
            pkey[o + e] = FLT_MAX;
            pid[o + e] = -1;
          }
          const float tl = fminf(qcut[gq[qb]], li[qb][KR - 1] >= 0 ? lk[qb][KR - 1] : FLT_MAX);
          tq[qb] = gq[qb] < nqa ? tl : -FLT_MAX;
          dc[qb] = dcount[g];
          asm volatile("" ::"v"(tq[qb]), "v"(dc[qb]));
        }
        if constexpr (EL == FILTER_I8) {
          set_factor_bounds(tsw);
          set_Tq();
        }
      }
    };

    AccT<EL> acc[4][2];
    // fragments of one sub-step: A (database rows) x4, B (queries) x2
    uint4 fa0[4], fb0[2], fa1[4], fb1[2];
    auto rd = [&](int buf, int s2, uint4 (&fa)[4], uint4 (&fb)[2]) {
      const char* base = smem + buf * 2 * kStepB;
      const int co = ((2 * s2 + h) ^ fsw) * 16;
      const char* cX = base + (128 * wr + c32) * 64 + co;
      const char* cQ = base + kStepB + (64 * wq + c32) * 64 + co;
      if constexpr (!VS_X1_P(2)) {
        fb[0] = *(const uint4*)cQ;
        fb[1] = *(const uint4*)(cQ + 32 * 64);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) fa[rb] = *(const uint4*)(cX + rb * 32 * 64);
      } else {
        auto opq = [](uint4& u) { asm volatile("" : "+v"(u.x), "+v"(u.y), "+v"(u.z), "+v"(u.w)); };
        asm volatile("" ::"v"(cX), "v"(cQ));
        opq(fb[0]);
        opq(fb[1]);
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) opq(fa[rb]);
      }
    };
    auto mfma_rb = [&](int rb, const uint4 (&fa)[4], const uint4 (&fb)[2]) {
      acc[rb][0] = mfma_blk<EL>(fa[rb], fb[0], acc[rb][0]);
      acc[rb][1] = mfma_blk<EL>(fa[rb], fb[1], acc[rb][1]);
    };
    // the first sub-step of a tile: C = 0 (inline constant), no clearing pass
    auto mfma_rb_first = [&](int rb, const uint4 (&fa)[4], const uint4 (&fb)[2]) {
      const AccT<EL> z = {};
      acc[rb][0] = mfma_blk<EL>(fa[rb], fb[0], z);
      acc[rb][1] = mfma_blk<EL>(fa[rb], fb[1], z);
    };
    // the four LDS-DMA pieces of the load cursor's step, one at a time
    auto stage_piece = [&](int i) {
      // uniform bases (the piece's permuted 16-row group of the load tile, the
      // query tile's) + per-lane offsets below 256 rows
      const char* xbase = XH + ((int64_t)lt * nksteps + lk_) * kStepB +
                          (uint32_t)((32 * w + 16 * (i >> 1)) ^ xhi) * 64u;
      const char* qbase = qtile + (int64_t)lk_ * kStepB + (uint32_t)(16 * (i >> 1)) * 64u;
      const uint32_t lx = lds0 + (uint32_t)lbuf * (2 * kStepB) + (uint32_t)(2 * w) * 1024u;
      if constexpr (!VS_X1_P(1)) {
        if ((i & 1) == 0) {
          if constexpr (!VS_X1_P(16))
            glds16(xbase, xlane, __builtin_amdgcn_readfirstlane(lx + (i >> 1) * 1024u));
        } else {
          if constexpr (!VS_X1_P(32))
            glds16(qbase, soff, __builtin_amdgcn_readfirstlane(lx + kStepB + (i >> 1) * 1024u));
        }
      } else {
        asm volatile("" ::"v"(xlane), "v"(soff), "s"(xbase), "s"(qbase), "s"(lx));
      }
    };
    auto advance_cursor = [&]() {
      if (ls + 1 < nsteps) {
        ++ls;
        if constexpr (kSeg) {  // a tile change rebuilds them below
          xstep += kStepB;
          qstep += kStepB;
        }
        if (++lk_ == nksteps) {
          lk_ = 0;
          set_xoff(++lt);
          if constexpr (kSeg) set_step_ptrs();
        }
      }
      lbuf = lbuf + 1 == NBUF ? 0 : lbuf + 1;
    };
    // the four pieces of the load cursor's step in stage_piece's order (X
    // group 0, Q rows 0-15, X group 1, Q rows 16-31); M0 saved once, set per
    // piece (one wait state before each LDS-DMA reads it).  No instruction
    // offsets: an LDS-DMA adds its offset to the LDS address as well.
    auto stage_step = [&]() {
      if constexpr (!kSeg || (VS_X1_PROBE & (1 | 16 | 32)) != 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) stage_piece(i);
      } else {
        const uint32_t lx = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)lbuf * (2 * kStepB) +
                                                           (uint32_t)(2 * w) * 1024u);
        uint32_t keep;
        asm volatile(
            "s_mov_b32 %0, m0\n\t"
            "s_mov_b32 m0, %4\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %1, %5\n\t"
            "s_add_u32 m0, %4, 0x4000\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %3, %6\n\t"
            "s_add_u32 m0, %4, 0x400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %2, %5\n\t"
            "s_add_u32 m0, %4, 0x4400\n\ts_nop 0\n\t"
            "global_load_lds_dwordx4 %7, %6\n\t"
            "s_mov_b32 m0, %0"
            : "=&s"(keep)
            : "v"(xl0), "v"(xl2), "v"(soff), "s"(lx), "s"(xstep), "s"(qstep), "v"(soff + 1024u)
            : "memory");
        static_assert(kStepB == 0x4000, "stage_step's M0 offsets");
      }
    };
#if VS_X1_STAMP
    unsigned long long ecnt[kStampCnt] = {0, 0, 0};  // only [0] (wave level) is kept
    unsigned long long sg[kStampSeg] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long tA = 0, tB = 0, eA = 0, eB = 0;
#define VS_X1_COUNT(i, v) (ecnt[i] += (v))
#define VS_X1_EMARK(i) (eB = stamp_now(), sg[i] += eB - eA, eA = eB)
#else
#define VS_X1_COUNT(i, v) ((void)0)
#define VS_X1_EMARK(i) ((void)0)
#endif
    auto epilogue = [&](int t, auto dm_tag) {
      // dm_tag: a dump launch's epilogue (also the dump part of a hybrid one)
      constexpr bool DM = decltype(dm_tag)::value;
      // a block's admission limit: the list's last entry, or the floor
      auto lim = [&](int qb) -> float {
        if constexpr (DM) return tq[qb];
        else return lk[qb][KL - 1];
      };
      // uniform: every row of the tile exists and none is excluded
      const bool plain = self0 < 0 && !qrow && (t + 1) * kT <= ntotal;
      const int f = tile_perm(t);
      const int fh = (4 * h) ^ (f & 0x04);
      // slot 128 wr + 32 rb + 8 jj + 4 h + e holds row t kT + (slot ^ f); the
      // slot's fields are disjoint bits, so the XOR splits into a uniform part
      // (wr, rb, jj) and one lane part (h), and f leaves the low two bits (e)
      auto rowof = [&](int rb, int jj) {
        return t * kT + ((128 * wr + 32 * rb) ^ (f & 0xE0)) + ((8 * jj) ^ (f & 0x18)) + fh;
      };
      // Phase 1: the candidate rows of every (rb, qb) block, one bit per block,
      // against each block's limit before any insertion of this tile (a list's
      // last entry only tightens, so the bits are a superset).
      //  * int8: a row's score fl(fl(float(sum)) * fl(f_q * f_x)) is monotone
      //    in the sum and in f_x (factors >= 0), so with the lane's largest
      //    factor over its 16 rows (xgmax: the maximum per 32-row group and
      //    bit 2 of the row, a SCALAR load) a row can beat the limit only if
      //    its int32 sum exceeds one integer threshold per block (i8_threshold):
      //    a maximum and one compare;
      //  * bf16 inner product: the key is -sum, exactly: a maximum and a compare;
      //  * bf16 L2 / cosine: every row (the key needs the row's norm).
      uint32_t pass = 0;
      float fmx[4];  // int8: the lane's factor bound per row block
#if VS_X1_STAMP
      if constexpr (EL == FILTER_I8) eA = stamp_now();
#endif
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
        fmx[rb] = 0.0f;
        if constexpr (EL == FILTER_I8 && !DM) {
          const int grp = (t * kT + ((128 * wr + 32 * rb) ^ (f & 0xE0))) >> 5;  // uniform
          const float g0 = xgmax[2 * grp], g1 = xgmax[2 * grp + 1];
          fmx[rb] = (fh & 4) ? g1 : g0;
        }
      }
#if VS_X1_STAMP
      if constexpr (EL == FILTER_I8) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) asm volatile("" ::"v"(fmx[rb]));
        VS_X1_EMARK(7);
      }
#endif
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          const float last = lim(qb);
          bool p;
          if constexpr (EL == FILTER_I8 && DM) {
            int amax = acc[rb][qb][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) amax = max(amax, acc[rb][qb][r]);
            p = amax > Tq[qb];
          } else if constexpr (EL == FILTER_I8) {
            const float c = qsc[qb] * fmx[rb];
            if (c > 0.0f && -last >= 0.0f) {
              int amax = acc[rb][qb][0];
#pragma unroll
              for (int r = 1; r < 16; ++r) amax = max(amax, acc[rb][qb][r]);
              p = amax > i8_threshold(-last, c);
            } else {
              p = c > 0.0f || -0.0f < last;
            }
          } else if constexpr (MODE == MODE_IP) {
            float amax = acc[rb][qb][0];
#pragma unroll
            for (int r = 1; r < 16; ++r) amax = fmaxf(amax, acc[rb][qb][r]);
            p = -amax < last;  // NaN sums never enter
          } else {
            p = true;
          }
          pass |= (uint32_t)p << (2 * rb + qb);
        }
      }
      VS_X1_EMARK(6);
      if constexpr (VS_X1_P(128)) {
        asm volatile("" ::"v"(pass));
        pass = 0;
      }
      if constexpr (DM) {
        // Dump launch: every row of a block that passed whose sum clears the
        // limit (int8: above the launch's integer threshold; bf16: -sum below
        // the limit) goes to the lane list's
        // next slot as (row, raw sum): one 8-B store per candidate row (the
        // stores queue behind the DMA pieces like everything in the vector
        // memory path: a whole block's 16 sums took five stores and ~4 % of a
        // C3 step, profiles/r04f/stamp_c3_dump.txt).  A list past its dR slots
        // counts on (the replay fails its query).
        // (a block, not an early return: one exit keeps the step loop's
        // branch to the epilogue a single compare)
        if (__ballot(pass != 0) != 0) {  // uniform: rare
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) {
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            if (pass & (1u << (2 * rb + qb))) {
              const float last = lim(qb);
              uint32_t cm = 0;
              if constexpr (EL == FILTER_I8) {
#pragma unroll
                for (int r = 0; r < 16; ++r) cm |= (uint32_t)(acc[rb][qb][r] > Tq[qb]) << r;
              } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) cm |= (uint32_t)(-acc[rb][qb][r] < last) << r;
              }
              while (cm) {
                const int bi = __builtin_ctz(cm);
                cm &= cm - 1;
                // rows past the corpus (the last tile's zero padding, whose sums
                // of 0 clear a floor above 0) take no slot
                const int row = rowof(rb, bi >> 2) + (bi & 3);
                if (!plain && !(row < ntotal && row != selfrow[qb])) continue;
                const int c = dc[qb]++;
                if (c < dR) {
                  int sum;
                  if constexpr (EL == FILTER_I8) sum = sel16i(acc[rb][qb], bi);
                  else sum = __float_as_int(sel16(acc[rb][qb], bi));
                  // slot-major (slot c of every list together): the replay's
                  // threads, one per list, read their c-th slots coalesced
                  const int64_t slot = (int64_t)c * ((int64_t)nqt * kT * P) + (int64_t)gq[qb] * P + pl;
                  *(i32x2*)(dslot + slot * 2) = i32x2{row, sum};
                }
              }
            }
          }
        }
        }
        VS_X1_EMARK(8);
      } else {
      // Phases 2 and 3 per half tile (rb pair): the per-row values (int8
      // factors; bf16 L2 / cosine norms) of the lane's 32 rows, when any lane of
      // the wave has a candidate in the pair — eight 16-B loads in ONE asm
      // statement that also retires them (vmcnt(0), which drains the LDS-DMA
      // pieces in flight too: twice per tile at most; loads the compiler sees
      // would get a vmcnt counted without the DMA pieces, and its waits would
      // leak into the loop) — then the exact keys of the candidates, admitted
      // with key < the list's last entry (a row tied with it is left out even
      // when its label is lower: the lists are candidate pools, and the
      // verification only needs every row outside them to have an approximate
      // key >= its list's final last entry, which this keeps); list_insert
      // orders the admitted rows lexicographically.  The fragment registers
      // are dead here (reloaded by the next load segment).
      constexpr bool kRows = EL == FILTER_I8 || MODE == MODE_L2 || MODE == MODE_COS;
      // row blocks per load group: 2 under the segmented schedule; 1 under the
      // round-2 schedule, whose next-step fragments stay live across the
      // epilogue (registers)
      constexpr int G = x1_sched(EL, DUMP, HYB) != 1 ? 2 : 1;
#pragma unroll
      for (int hp = 0; hp < 4 / G; ++hp) {
        f32x4 rv[G][4];
#pragma unroll
        for (int r2 = 0; r2 < G; ++r2)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) rv[r2][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
        const uint32_t any = (pass >> (2 * G * hp)) & ((1u << (2 * G)) - 1u);
        if (__ballot(any != 0) == 0) continue;  // uniform
        if constexpr (kRows) {
          const float* src = EL == FILTER_I8 ? xs : xaux;
          if constexpr (G == 2) {
            const float* a[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) a[q] = src + rowof(2 * hp + (q >> 2), q & 3);
            asm volatile(
                "global_load_dwordx4 %0, %8, off\n\tglobal_load_dwordx4 %1, %9, off\n\t"
                "global_load_dwordx4 %2, %10, off\n\tglobal_load_dwordx4 %3, %11, off\n\t"
                "global_load_dwordx4 %4, %12, off\n\tglobal_load_dwordx4 %5, %13, off\n\t"
                "global_load_dwordx4 %6, %14, off\n\tglobal_load_dwordx4 %7, %15, off\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(rv[0][0]), "=&v"(rv[0][1]), "=&v"(rv[0][2]), "=&v"(rv[0][3]),
                  "=&v"(rv[G - 1][0]), "=&v"(rv[G - 1][1]), "=&v"(rv[G - 1][2]), "=&v"(rv[G - 1][3])
                : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),
                  "v"(a[7])
                : "memory");
          } else {
            const float* a[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) a[q] = src + rowof(hp, q);
            asm volatile(
                "global_load_dwordx4 %0, %4, off\n\tglobal_load_dwordx4 %1, %5, off\n\t"
                "global_load_dwordx4 %2, %6, off\n\tglobal_load_dwordx4 %3, %7, off\n\t"
                "s_waitcnt vmcnt(0)"
                : "=&v"(rv[0][0]), "=&v"(rv[0][1]), "=&v"(rv[0][2]), "=&v"(rv[0][3])
                : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3])
                : "memory");
          }
          __builtin_amdgcn_sched_barrier(0);
          VS_X1_COUNT(0, 1);  // uniform: a scalar count
        }
#pragma unroll
        for (int r2 = 0; r2 < G; ++r2) {
          const int rb = G * hp + r2;
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            if (!(pass & (1u << (2 * rb + qb)))) continue;
            uint32_t cm = 0;
            if constexpr ((MODE == MODE_L2 || MODE == MODE_COS) && EL != FILTER_I8) {
              // every row is a candidate: keys first, admission mask from them
              f32x16 key;
#pragma unroll
              for (int jj = 0; jj < 4; ++jj)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  const float v = acc[rb][qb][jj * 4 + e];
                  key[jj * 4 + e] = MODE == MODE_L2 ? l2_from_ip(qa[qb], rv[r2][jj][e], v)
                                                    : -(v * (qa[qb] * rv[r2][jj][e]));
                }
              const float last = lim(qb);
              cm = 0;
#pragma unroll
              for (int r = 0; r < 16; ++r) cm |= (uint32_t)(key[r] < last) << r;
              if (!plain) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                  const int row = rowof(rb, r >> 2) + (r & 3);
                  if (!(row < ntotal && row != selfrow[qb])) cm &= ~(1u << r);
                }
              }
              while (cm) {
                const int bi = __builtin_ctz(cm);
                cm &= cm - 1;
                const int row = rowof(rb, bi >> 2) + (bi & 3);
                list_insert<KR, int>(lk[qb], li[qb], sel16(key, bi), row);
              }
            } else {
              // the block's candidate rows (int8: sum above the block's integer
              // threshold; bf16: -sum below the last entry), then one at a time:
              // the exact key of the row and its admission
              const float last = lim(qb);
              if constexpr (EL == FILTER_I8) {
                const float c = qsc[qb] * fmx[rb];
                const int T = (c > 0.0f && -last >= 0.0f) ? i8_threshold(-last, c) : INT_MIN;
#pragma unroll
                for (int r = 0; r < 16; ++r) cm |= (uint32_t)(acc[rb][qb][r] > T) << r;
              } else {
#pragma unroll
                for (int r = 0; r < 16; ++r) cm |= (uint32_t)(-acc[rb][qb][r] < last) << r;
              }
              while (cm) {
                const int bi = __builtin_ctz(cm);
                cm &= cm - 1;
                const int row = rowof(rb, bi >> 2) + (bi & 3);
                float key;
                if constexpr (EL == FILTER_I8)
                  key = x1_key<EL>(sel16i(acc[rb][qb], bi), qsc[qb], sel4x4(rv[r2], bi));
                else
                  key = -sel16(acc[rb][qb], bi);
                const bool ok = (plain || (row < ntotal && row != selfrow[qb])) && key < lim(qb);
                if (ok) list_insert<KR, int>(lk[qb], li[qb], key, row);
              }
            }
          }
        }
        VS_X1_EMARK(8);
      }
      }
    };

    constexpr int kSched = x1_sched(EL, DUMP, HYB);
    if constexpr (kSched == 1) {

    // prologue: steps 0 .. D-1 in flight, retire step 0, read its first fragments
#pragma unroll
    for (int i = 0; i < D; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) stage_piece(j);
      advance_cursor();
    }
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // step 0 of the D in flight
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    rd(0, 0, fa0, fb0);
    int buf = 0;
    // The instruction order inside a step is pinned with sched_barrier(0): hipcc
    // would otherwise move the MFMAs across the barrier and the fragment reads
    // next to their first use, undoing the half-step lookahead.
    // Stagger: waves 4-7 take the step's barrier at its start instead of its
    // middle, so they run half a step behind their SIMD partners (the LDS-DMA
    // issue of one wave beside the other's MFMAs).  Every condition above
    // still holds for them: they retire DMA(s+1) before barrier s and read
    // image s+1 only after it, and their last reads of image s-1 are consumed
    // before barrier s, after which DMA(s+D) may overwrite it.
    const bool lag = w >= 4;
#if VS_X1_STAMP
    tA = stamp_now();
#define VS_X1_MARK1(i) (tB = stamp_now(), sg[i] += tB - tA, tA = tB)
#else
#define VS_X1_MARK1(i) ((void)0)
#endif
    // one step; `first` as in the segmented schedule's seg_step (peeled)
    auto s1_step = [&](auto first_tag) {
      constexpr bool first = decltype(first_tag)::value;
      const int nbuf = buf + 1 == NBUF ? 0 : buf + 1;
      // this wave's pieces of step s+1: the steps s+2 .. s+D-1 stay in flight
      // (the lagging waves wait before this step's first pieces, the others
      // after them)
      if (lag) {  // uniform
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
      // first half: sub-step 0 (fragments read during the previous step), with
      // the sub-step 1 reads of this step's image issued behind two MFMAs
      if constexpr (first) {  // a tile's first step starts its accumulators
        mfma_rb_first(0, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        rd(buf, 1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rb_first(1, fa0, fb0);
        mfma_rb_first(2, fa0, fb0);
        mfma_rb_first(3, fa0, fb0);
      } else {
        mfma_rb(0, fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        rd(buf, 1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rb(1, fa0, fb0);
        mfma_rb(2, fa0, fb0);
        mfma_rb(3, fa0, fb0);
      }
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK1(0);
      // retire step s+1 (this wave's pieces); the younger D-2 steps stay in flight
      if (!lag) {  // uniform
        if constexpr (!VS_X1_P(64)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        if constexpr (!VS_X1_P(4)) __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK1(1);
      // second half: next step's sub-step 0 reads first (their latency hides under
      // this half's MFMAs), then sub-step 1's MFMAs with the LDS-DMA of step s+D
      // (into the image of step s-1, which every wave has finished) between them
      rd(nbuf, 0, fa0, fb0);  // past the end: a harmless read of a stale image
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        mfma_rb(i, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        stage_piece(i);
        __builtin_amdgcn_sched_barrier(0);
      }
      advance_cursor();
      VS_X1_MARK1(3);
      VS_X1_MARK1(5);
      buf = nbuf;
    };
    // tiles [ta, tb) with the epilogue of kind DM (a hybrid launch: its list
    // part, then its dump part — two loops, so the lists are dead in the
    // second)
    auto s1_tiles = [&](int ta, int tb, auto dm_tag) {
      for (int t = ta; t < tb; ++t) {
        s1_step(std::true_type{});
        for (int k = 1; k < nksteps; ++k) s1_step(std::false_type{});
        if constexpr (!VS_X1_P(8)) {
          epilogue(t, dm_tag);
        } else {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) asm volatile("" ::"v"(acc[rb][qb]));
        }
        VS_X1_MARK1(5);
      }
    };
    if constexpr (HYB) {
      s1_tiles(t0, tsw, std::false_type{});
      to_dump_mode();
      s1_tiles(tsw, t1, std::true_type{});
    } else {
      s1_tiles(t0, t1, std::integral_constant<bool, DUMP>{});
    }
#undef VS_X1_MARK1
    } else {
    // Segmented schedule: every step of a wave is a LOAD segment (the step's 12
    // fragment reads, the 4 LDS-DMA pieces of step s+3, the wait for this
    // wave's pieces of step s+1) and a MATRIX segment (the step's 16 MFMAs),
    // each closed by a barrier.  Waves 4-7 run one barrier behind waves 0-3,
    // so on every SIMD one wave's load segment — whose DMA issue stalls that
    // wave for ~100-185 cycles per piece (MI355X_MICROARCH.md, LDS-DMA piece
    // issue cost) — runs beside its partner's matrix segment, and no wave's
    // MFMA stream is cut by its own DMA issue (the 8-phase GEMM template's
    // pairing, cdna_hip_programming.md).  3 steps in flight over a ring of 5
    // images: the image a DMA refills was read two barriers earlier by every
    // wave (reads retired by the lgkmcnt wait that opens the reader's matrix
    // segment); an image is read only after the barrier that follows every
    // wave's counted wait for its pieces.
    // (4 steps in flight, each load segment closed by an lgkmcnt(0) so the
    // image a DMA refills could be the one read a barrier earlier: C3 70.2k vs
    // 70.8k queries/s, C2 -3 %, C4 -2 %: not shipped.  The query fragments
    // loaded straight into registers, one step ahead, instead of through LDS
    // (half the DMA pieces, two thirds of the fragment reads): C3 +0.3 %, so
    // the cost is the bytes entering the CU, not the LDS path; s_setprio on
    // either half: -0.1 %; profiles/r04n/ab_qreg_prio.txt: not shipped)
    static_assert(NBUF == 5, "segmented schedule: 3 steps in flight over 5 images");
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      stage_step();
      advance_cursor();
    }
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's pieces of step 0
    __builtin_amdgcn_s_barrier();
    const bool lag = w >= 4;
    if (lag) __builtin_amdgcn_s_barrier();  // uniform: one barrier behind
    int buf = 0;
#if VS_X1_STAMP
    tA = stamp_now();
#define VS_X1_MARK(i) (tB = stamp_now(), sg[i] += tB - tA, tA = tB)
#else
#define VS_X1_MARK(i) ((void)0)
#endif
    // One step; `first` (a tile's first step, which starts its accumulators)
    // is a compile-time tag: the loops below peel it, so a step carries no
    // branch on its position in the tile.
    auto seg_step = [&](auto first_tag) {
      constexpr bool first = decltype(first_tag)::value;
      __builtin_amdgcn_sched_barrier(0);
      rd(buf, 0, fa0, fb0);
      rd(buf, 1, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
#if !VS_X1_SEGDMA
      stage_step();
      advance_cursor();
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK(0);
      // this wave's pieces of step s+1 (the younger steps stay in flight)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#else
      VS_X1_MARK(0);
      // this wave's pieces of step s+1; step s+2's (issued in the previous
      // matrix segment) stay in flight
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#endif
      VS_X1_MARK(1);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK(2);
#if !VS_X1_SEGDMA
      if constexpr (first) {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) mfma_rb_first(rb, fa0, fb0);
      } else {
#pragma unroll
        for (int rb = 0; rb < 4; ++rb) mfma_rb(rb, fa0, fb0);
      }
#pragma unroll
      for (int rb = 0; rb < 4; ++rb) mfma_rb(rb, fa1, fb1);
#else
      {
        // step s+3's pieces into the image of step s-2 (read two barriers ago
        // by every wave, as in the load segment's placement), one per four MFMAs
        const uint32_t lx = __builtin_amdgcn_readfirstlane(lds0 + (uint32_t)lbuf * (2 * kStepB) +
                                                           (uint32_t)(2 * w) * 1024u);
        auto piece = [&](int j, uint32_t m0v, uint32_t voff, const char* sbase) {
          if constexpr (!kSeg) {  // the bf16 L2 / cosine kernels: no step pointers
            stage_piece(j);
            return;
          }
          uint32_t keep;
          asm volatile(
              "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\t"
              "global_load_lds_dwordx4 %2, %3\n\ts_mov_b32 m0, %0"
              : "=&s"(keep)
              : "s"(m0v), "v"(voff), "s"(sbase)
              : "memory");
        };
        static_assert(kStepB == 0x4000, "piece offsets");
        if constexpr (first) {
          mfma_rb_first(0, fa0, fb0);
          mfma_rb_first(1, fa0, fb0);
        } else {
          mfma_rb(0, fa0, fb0);
          mfma_rb(1, fa0, fb0);
        }
        __builtin_amdgcn_sched_barrier(0);
        piece(0, lx, xl0, xstep);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (first) {
          mfma_rb_first(2, fa0, fb0);
          mfma_rb_first(3, fa0, fb0);
        } else {
          mfma_rb(2, fa0, fb0);
          mfma_rb(3, fa0, fb0);
        }
        __builtin_amdgcn_sched_barrier(0);
        piece(1, lx + 0x4000u, soff, qstep);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rb(0, fa1, fb1);
        mfma_rb(1, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        piece(2, lx + 0x400u, xl2, xstep);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rb(2, fa1, fb1);
        mfma_rb(3, fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
        piece(3, lx + 0x4400u, soff + 1024u, qstep);
        __builtin_amdgcn_sched_barrier(0);
        advance_cursor();
      }
#endif
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK(3);
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      VS_X1_MARK(4);
      VS_X1_MARK(5);
      buf = buf + 1 == NBUF ? 0 : buf + 1;
    };
    auto seg_tiles = [&](int ta, int tb, auto dm_tag) {
      for (int t = ta; t < tb; ++t) {
        seg_step(std::true_type{});
        for (int k = 1; k < nksteps; ++k) seg_step(std::false_type{});
        // the tile's epilogue, beside the partner's matrix segment
        if constexpr (!VS_X1_P(8)) {
          epilogue(t, dm_tag);
        } else {
#pragma unroll
          for (int rb = 0; rb < 4; ++rb)
#pragma unroll
            for (int qb = 0; qb < 2; ++qb) asm volatile("" ::"v"(acc[rb][qb]));
        }
        VS_X1_MARK(5);
      }
    };
    if constexpr (HYB) {
      seg_tiles(t0, tsw, std::false_type{});
      to_dump_mode();
      seg_tiles(tsw, t1, std::true_type{});
    } else {
      seg_tiles(t0, t1, std::integral_constant<bool, DUMP>{});
    }
    if (!lag) __builtin_amdgcn_s_barrier();  // the lagging waves' extra one
#undef VS_X1_MARK
    }
#if VS_X1_STAMP
    {  // vector atomics; the counts are summed over the lanes
      const int grp = w >= 4 ? 1 : 0;
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < kStampSeg; ++i)
          atomicAdd(&g_x1_stamps[grp * (kStampSeg + kStampCnt) + i], sg[i]);
        atomicAdd(&g_x1_stamps[2 * (kStampSeg + kStampCnt) + grp], (unsigned long long)nsteps);
      }
      if (lane == 0)
        atomicAdd(&g_x1_stamps[grp * (kStampSeg + kStampCnt) + kStampSeg], ecnt[0]);
    }
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // drain before the workgroup exits
  }

  // the list offsets are recomputed from the lane id here (not kept live
  // across the main loop: registers)
  const int ln = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  const int pl0 = sp * 4 + wr * 2 + (ln >> 5);
  // (a hybrid launch stored its lists at the switch, which every workgroup
  // with a tile reaches: its lists are dead past it, registers)
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t g = (int64_t)(qt * kT + 64 * wq + 32 * qb + (ln & 31)) * P + pl0;
    if (DUMP || (HYB && t1 > t0)) {
      dcount[g] = dc[qb];
    } else if (HYB) {  // no tile: empty lists
      const int64_t o = g * KP;
      for (int e = 0; e < KP; ++e) {
        pkey[o + e] = FLT_MAX;
        pid[o + e] = -1;
      }
    } else {
      const int64_t o = g * KP;
#pragma unroll
      for (int e = 0; e < KR; ++e) {
        pkey[o + e] = lk[qb][e];
        pid[o + e] = li[qb][e];
      }
      for (int e = KR; e < KP; ++e) {
        pkey[o + e] = FLT_MAX;
        pid[o + e] = -1;
      }
    }
  }
}

// The replay of a segment of dump launches: one thread per lane list (query
// q, list pl = 4 sp + 2 wr + h).  The list as the previous launches left it,
// then every row dumped since in dump order (the order the lane met them:
// tiles ascending, launch after launch) with the key the list epilogue
// computes (x1_key, the same expression) and the same admission: key <
// min(last entry, cut), the row inside the corpus and not the query's own; the
// count restarts at zero for the next segment.  A list with more dumps than
// slots lost some: its query's cut becomes -FLT_MAX, which fails both checks
// of the verification (the query goes to the next stage) and stops the
// query's dumps.
template <int KR, int EL>
__global__ __launch_bounds__(256) void x1_replay_kernel(
    int* __restrict__ dcount, const int* __restrict__ dslot, float* __restrict__ pkey,
    int* __restrict__ pid, int P, int KP, int nqa, const float* __restrict__ qs,
    const float* __restrict__ xs, int64_t self0, int ntotal, int dR, int64_t nl,
    float* __restrict__ qcut, unsigned long long* __restrict__ stats) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int cnt = i < (int64_t)nqa * P ? dcount[i] : 0;
  {  // statistics: one atomic per wave
    unsigned long long a = (unsigned long long)cnt, b = cnt > dR ? 1ull : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
      a += __shfl_xor(a, o);
      b += __shfl_xor(b, o);
    }
    if ((threadIdx.x & 63) == 0 && a && stats) {
      atomicAdd(stats, a);
      if (b) atomicAdd(stats + 1, b);
    }
  }
  if (cnt == 0) return;
  dcount[i] = 0;  // the next segment's dumps start at slot 0
  const int q = (int)(i / P);
  if (cnt > dR) {
    qcut[q] = -FLT_MAX;
    return;
  }
  const float cut = qcut[q];
  const float qsc = EL == FILTER_I8 ? qs[q] : 0.0f;
  const int selfrow = self0 >= 0 ? (int)(self0 + q) : -1;
  static_assert(KR % 4 == 0, "lane lists move as 16-B pieces");
  float lk[KR];
  int li[KR];
  const int64_t o = i * KP;  // KP: a multiple of 4 (launch_x1_replay)
#pragma unroll
  for (int e = 0; e < KR; e += 4) {
    const f32x4 kv = *(const f32x4*)(pkey + o + e);
    const int4 iv = *(const int4*)(pid + o + e);
    lk[e] = kv.x, lk[e + 1] = kv.y, lk[e + 2] = kv.z, lk[e + 3] = kv.w;
    li[e] = iv.x, li[e + 1] = iv.y, li[e + 2] = iv.z, li[e + 3] = iv.w;
  }
  // the list's slots c = 0 .. cnt-1 at dslot[c * nl + i] (slot-major), eight
  // at a time: their loads, then their rows' factors, then the admissions in
  // dump order (independent loads in flight together instead of a chain)
  const i32x2* sl = (const i32x2*)dslot + i;
  constexpr int kB = 8;
  for (int c0 = 0; c0 < cnt; c0 += kB) {
    i32x2 e[kB];
    float fx[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) e[j] = c0 + j < cnt ? sl[(int64_t)(c0 + j) * nl] : i32x2{-1, 0};
#pragma unroll
    for (int j = 0; j < kB; ++j)
      fx[j] = EL == FILTER_I8 && e[j][0] >= 0 && e[j][0] < ntotal ? xs[e[j][0]] : 0.0f;
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int row = e[j][0];
      if (!(row >= 0 && row < ntotal && row != selfrow)) continue;
      const float key = x1_key<EL>(e[j][1], qsc, fx[j]);
      if (key < fminf(lk[KR - 1], cut)) list_insert<KR, int>(lk, li, key, row);
    }
  }
#pragma unroll
  for (int e = 0; e < KR; e += 4) {
    *(f32x4*)(pkey + o + e) = f32x4{lk[e], lk[e + 1], lk[e + 2], lk[e + 3]};
    *(int4*)(pid + o + e) = make_int4(li[e], li[e + 1], li[e + 2], li[e + 3]);
  }
}

// Query tiles per XCD of the blocked grid (env VS_X1_QG for A/B; default 4).
static int x1_qg() {
  static const int v = [] {
    const char* e = getenv("VS_X1_QG");
    const int q = e ? atoi(e) : 0;
    return q > 0 ? q : 4;
  }();
  return v;
}

static hipError_t launch_qcut(const X1Args& a, Partials part, hipStream_t st);

// XCD rounds of query-tile groups for grids of more than 8 groups (env
// VS_X1_XCDG=0 turns them off, for A/B; read at every search)
static bool x1_group_rounds() {
  const char* e = getenv("VS_X1_XCDG");
  return !e || atoi(e) != 0;
}

// Hybrid first launches (env VS_X1_HYB=1, read at every search; off by
// default): for a workgroup with at least kHybMinTiles tiles in the launch (its
// list part, a quarter of them, then sees >= 4 tiles: 256 rows per lane list).
// Measured against list first launches on one box (profiles/r05j): C2 348.5k
// vs 397.6k queries/s (the single launch's replay and dump stores cost more
// than the list epilogue they replace), C3 76.4k vs 76.7k, clustered C3 equal:
// kept as an exact, tested alternative, not the default.
constexpr int kHybMinTiles = 16;
// split passes: a list launch over the first 1/8 of every workgroup's tiles
// (x1_split_den; C2 on one box, profiles/r05m: 426k queries/s at 1/8, 416k at
// 1/4, 410k as one list launch)
constexpr int kX1SplitDen = 8;
static bool x1_hybrid_on() {
  const char* e = getenv("VS_X1_HYB");
  return e && atoi(e) != 0;
}

// Database tiles per workgroup per launch for a pass of per_block tiles per
// workgroup: 64, or 32 for a pass that can dump and has 128-192 tiles per
// workgroup, which 64-tile launches would cut into fewer than 4 (no dumps) and
// 32-tile ones into 4-6 (one list launch, the rest dumps): a 1.25M-row shard
// at 16 query tiles (C3 over 8 GPUs), 153 tiles: 435k vs 423k queries/s; with
// 305 tiles (2.5M rows) and at C3, 32-tile launches lose 2 % and 1 %
// (profiles/r04t/ab_chunk.txt).  Env VS_X1_CHUNK_TILES overrides both (read at
// every search: A/B runs, and tests that need multi-launch passes on small
// indexes).
// (round 6: 40-tile launches there, four of them for the 1.25M-row rank —
// one list launch, three dumps — instead of five 32-tile ones: 460.5k vs
// 447.6k / 451.6k queries/s, profiles/r06rc)
constexpr int kX1ShortChunkTiles = 40;
static int x1_chunk_tiles(int per_block, bool can_dump) {
  const char* e = getenv("VS_X1_CHUNK_TILES");
  const int v = e ? atoi(e) : 0;
  if (v > 0) return v;
  return can_dump && per_block >= 128 && per_block <= 3 * kX1ChunkTiles ? kX1ShortChunkTiles
                                                                        : kX1ChunkTiles;
}

// Split passes (env VS_X1_SPLIT=<den>, read at every search; 0 = off;
// default kX1SplitDen): a
// dump-capable pass too short for 4 launches (C2: one launch of 61 tiles per
// workgroup) runs as TWO launches, a list launch over the first 1/den of every
// workgroup's tiles and one dump launch over the rest, with the cut between
// them and one replay after: the dump launch's floor is min(cut, the list's
// last entry), so it stores a few rows per list where a hybrid launch's
// list-only floor stored ~24.
static int x1_split_den() {
  const char* e = getenv("VS_X1_SPLIT");
  return e ? std::max(0, atoi(e)) : kX1SplitDen;
}
// Segmented split passes (env VS_X1_SPLITSEG=1, read at every search; A/B):
// a split pass of den = 2^m parts (m >= 2) runs its dump part as m launches
// over parts [1, 2), [2, 4), .. [den / 2, den), a replay after each, so every
// segment doubles the rows seen and a lane list meets ~8 rows below its floor
// per segment however small the list launch's share (1 / den) is.
static bool x1_split_segments(int den) {
  const char* e = getenv("VS_X1_SPLITSEG");
  return e && atoi(e) != 0 && den >= 4 && (den & (den - 1)) == 0;
}
constexpr int kSplitMinTiles = 16;
// (default: the bf16 plane's passes only — clustered C3 +1.4 %, C3's int8
// pass -1 %, profiles/r05u)
// VS_X1_QUARTER=<F>: the list launch covers 1/F of the first chunk (0: off,
// 1: 1/4 as F = 4)
static int x1_first_den(int el) {
  const char* e = getenv("VS_X1_QUARTER");
  if (!e) return el == FILTER_BF16 ? 4 : 0;
  const int v = atoi(e);
  return v == 1 ? 4 : v >= 2 ? v : 0;
}

template <int KR, int MODE, int EL>
static hipError_t x1_launch(const X1Args& a, Partials part, hipStream_t st, int* ndispatch) {
  const int ntiles = (a.ntotal + kT - 1) / kT;
  const int nqt = a.nq_pad / kT;
  const int per_block = (ntiles + a.nsplit - 1) / a.nsplit;
  // A gathered later stage holds its few queries in the first query tile(s):
  // every XCD takes every query tile there (QG = nqt), so the working
  // workgroups of tile 0 spread over all XCDs instead of the 2 of 8 that QG = 4
  // gives it (clustered C3: 202 -> 151 ms per step, profiles/r02za).
  const int qg = a.qcount ? nqt : x1_qg() * (x1_group_rounds() ? 1 : -1);
  const bool dump = a.dump && x1_has_dump(MODE, EL) && !a.qcount && a.qcut && a.qbkey &&
                    a.qcut_m > 0 && a.dcount && a.dslot && a.dR > 0;
  const int chunk_tiles = x1_chunk_tiles(per_block, dump);
  // a gathered later stage (usually empty: its tiles exit at once) is one launch
  int nchunk = a.qcount ? 1 : std::max(1, (per_block + chunk_tiles - 1) / chunk_tiles);
  // Dump launches after the first: its lists set the cuts (x1_qcut), the rest
  // of the pass stores only the blocks below them, and x1_replay folds the
  // dumps into the lists between segments (below).  Passes of at least 4
  // launches (C3: 20) cut their launches as they are; a shorter one (C2) is
  // a split pass when VS_X1_SPLIT allows it (above); otherwise list launches
  // (C2 forced to 4 equal launches lost in round 4: 308k vs 394k queries/s,
  // profiles/r04a/r04d_sched_c2_cl_ab.txt).
  const int den = x1_split_den();
  const bool split = dump && nchunk < 4 && den >= 2 && per_block >= kSplitMinTiles;
  const bool cutting = dump && (nchunk >= 4 || split);  // x1_pass_dumps
  // Hybrid first launch (gemm_topk_x1<..., HYB>): a quarter of its tiles as a
  // list launch, the rest dumping below each list's own last entry; x1_replay
  // right after it.  It needs no cut, so a pass of fewer launches (C2: one)
  // dumps too, its later launches as dump launches below the lists' floors.
  const int tiles0 = (per_block + nchunk - 1) / nchunk;
  const bool hyb = dump && !split && x1_hybrid_on() && tiles0 >= kHybMinTiles;
  const bool later_dump = cutting || hyb;  // launches c > 0 are dump launches
  // the launches as part ranges [p0, p1) of nparts
  // Quarter-chunk list launches (env VS_X1_QUARTER=0/1; default: bf16 passes): a
  // cutting pass of nchunk launches lists only parts [0, 1) of 4 nchunk, then a
  // dump launch over [1, 4) and one launch per chunk.  The list launch runs at
  // ~2/3 of a dump launch's rate (a k = 60 pass of 5 chunks spent 15 of its
  // 58 ms in it, profiles/r05t), but cuts set from a quarter of the rows are
  // looser: C3 dumps 1.7x the rows, 76.5k vs 77.4k queries/s; k = 60 equal,
  // clustered +1.4 % (profiles/r05u).
  const int F = x1_first_den(EL);
  const bool quarter = cutting && !split && nchunk >= 4 && F >= 2 && per_block / (F * nchunk) >= 2;
  const bool sseg = split && x1_split_segments(den);
  int lg = 0;
  while ((1 << lg) < den) ++lg;
  const int nparts = split ? den : quarter ? F * nchunk : nchunk;
  const int nlaunch = sseg ? lg + 1 : split ? 2 : quarter ? nchunk + 1 : nchunk;
  const int64_t ldb = a.ld * filter_bytes(EL);
  if (a.qtile0 < 0) return hipErrorInvalidValue;
  for (int c = 0; c < nlaunch; ++c) {
    const int p0 = sseg    ? (c == 0 ? 0 : 1 << (c - 1))
                   : split   ? (c == 0 ? 0 : 1)
                   : quarter ? (c == 0 ? 0 : c == 1 ? 1 : F * (c - 1))
                             : c;
    const int p1 = sseg    ? (c == 0 ? 1 : 1 << c)
                   : split   ? (c == 0 ? 1 : den)
                   : quarter ? (c == 0 ? 1 : F * c)
                             : c + 1;
    // the timed span of this launch alone (the cut and replay kernels between
    // launches stay outside the spans); the first launch of a pass whose later
    // launches dump is timed apart ("<name>_list")
    if (a.timing)
      a.timing->begin(st, !(later_dump && nlaunch > 1) || c > 0, (double)(p1 - p0) / nparts);
    if (later_dump && c > 0) {
      if constexpr (x1_has_dump(MODE, EL))
        hipLaunchKernelGGL((gemm_topk_x1<KR, MODE, true, EL>), dim3(nqt * a.nsplit), dim3(512), 0,
                           st, (const char*)a.XH, a.xs, a.xaux, (const char*)a.QH, a.qs, a.qaux,
                           a.nqa, (int)(ldb / 64), a.ntotal, ntiles, a.nsplit, nqt, a.qtile0,
                           a.self0, a.qrow, a.qcount, p0, p1, nparts, part.KP, qg, part.key,
                           part.id, a.xgmax, a.xgmin, a.qcut, a.dcount, a.dslot, a.dR, a.qskip);
    } else if (hyb) {
      if constexpr (x1_has_dump(MODE, EL))
        hipLaunchKernelGGL((gemm_topk_x1<KR, MODE, false, EL, true>), dim3(nqt * a.nsplit),
                           dim3(512), 0, st, (const char*)a.XH, a.xs, a.xaux, (const char*)a.QH,
                           a.qs, a.qaux, a.nqa, (int)(ldb / 64), a.ntotal, ntiles, a.nsplit, nqt,
                           a.qtile0, a.self0, a.qrow, a.qcount, p0, p1, nparts, part.KP, qg,
                           part.key, part.id, a.xgmax, a.xgmin, a.qcut, a.dcount, a.dslot, a.dR, a.qskip);
    } else {
      hipLaunchKernelGGL((gemm_topk_x1<KR, MODE, false, EL>), dim3(nqt * a.nsplit), dim3(512), 0,
                         st, (const char*)a.XH, a.xs, a.xaux, (const char*)a.QH, a.qs, a.qaux,
                         a.nqa, (int)(ldb / 64), a.ntotal, ntiles, a.nsplit, nqt, a.qtile0,
                         a.self0, a.qrow, a.qcount, p0, p1, nparts, part.KP, qg, part.key,
                         part.id, a.xgmax, a.xgmin, nullptr, nullptr, nullptr, 0, a.qskip);
    }
    if (a.timing) a.timing->end(st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (hyb && c == 0) {  // the hybrid launch's dumps, before the cuts read the lists
      e = launch_x1_replay(a, part, st);
      if (e != hipSuccess) return e;
    }
    if (cutting && c == 0) {
      e = launch_qcut(a, part, st);
      if (e != hipSuccess) return e;
    }
    // Segments of dump launches end where the data seen doubles (after
    // launches 1, 3, 7, 15, ... and the last): a dump launch's threshold is
    // min(cut, list last entry at its start), and the replay between segments
    // lowers the last entries, so a lane list meets ~8 blocks below its own
    // floor per segment whatever the data (a top-8 list over n rows is beaten
    // by ~8 of the next n) — the cut alone is too wide when 2B spans
    // thousands of rows (C3: ~5k, 63 % of the lists out of 32 slots in one
    // segment, profiles/r04b).
    if (later_dump && c > 0 && (sseg || ((c + 1) & c) == 0 || c + 1 == nlaunch)) {
      e = launch_x1_replay(a, part, st);
      if (e != hipSuccess) return e;
    }
  }
  if (ndispatch) *ndispatch = nlaunch;
  return hipSuccess;
}

int x1_lane_len() { return 8; }
int x1_dump_slots() { return kDumpMaxR; }
bool x1_pass_dumps(int ntotal, int nsplit) {
  const int ntiles = (ntotal + kT - 1) / kT;
  const int per_block = (ntiles + nsplit - 1) / nsplit;
  const int ct = x1_chunk_tiles(per_block, true);
  const int nchunk = (per_block + ct - 1) / ct;
  return nchunk >= 4 || (x1_split_den() >= 2 && per_block >= kSplitMinTiles) ||
         (x1_hybrid_on() && (per_block + nchunk - 1) / nchunk >= kHybMinTiles);
}

hipError_t x1_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_x1_stamps), sizeof(g_x1_stamps));
  if (e == hipSuccess && reset) {
    unsigned long long z[kStampN] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_x1_stamps), z, sizeof(z));
  }
  return e;
}

template <int EL>
static hipError_t x1_dispatch(int mode, const X1Args& a, Partials part, hipStream_t st,
                              int* ndispatch) {
  switch (mode) {
    case MODE_IP:
      return x1_launch<8, MODE_IP, EL>(a, part, st, ndispatch);
    case MODE_L2:
      // int8: no L2 form (its key needs two per-row factors, which do not fit
      // the registers beside the accumulators); L2 indexes hold the bf16 plane
      if constexpr (EL == FILTER_I8) return hipErrorInvalidValue;
      else return x1_launch<8, MODE_L2, EL>(a, part, st, ndispatch);
    case MODE_COS:
      return x1_launch<8, MODE_COS, EL>(a, part, st, ndispatch);
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t launch_gemm_topk_x1(int mode, const X1Args& a, Partials part, hipStream_t st,
                               int* ndispatch) {
  // 64-B K-steps of plane rows padded to 64 elements; 256-query tiles; the
  // lists of a query are (split, row half, lane half)
  if (a.nq_pad % kT != 0 || a.ld % 64 != 0 || a.ld <= 0 || part.KP < x1_lane_len() ||
      part.P != 4 * a.nsplit || a.nsplit < 1 || a.ntotal <= 0)
    return hipErrorInvalidValue;
  if (a.filter == FILTER_I8) {
    if (!a.xs || !a.qs || !a.xgmax || !a.xgmin || a.ld > kI8MaxLd) return hipErrorInvalidValue;
    return x1_dispatch<FILTER_I8>(mode, a, part, st, ndispatch);
  }
  return x1_dispatch<FILTER_BF16>(mode, a, part, st, ndispatch);
}

bool x1_dump_applies(int mode, int filter) {
  return x1_has_dump(mode, filter) && (mode != MODE_COS || x1_cos_dump_on());
}

// The replay of launch_gemm_topk_x1's dumps (a no-op when the pass had none to
// make: the counts stay zero).
hipError_t launch_x1_replay(const X1Args& a, Partials part, hipStream_t st) {
  unsigned long long* stats = a.dstats;
  if (!a.dump || !a.dcount || a.nqa <= 0) return hipSuccess;
  if (part.KP < x1_lane_len() || part.KP % 4 != 0) return hipErrorInvalidValue;
  const int64_t n = (int64_t)a.nqa * part.P;
  const dim3 grid((unsigned)((n + 255) / 256));
  const int64_t nl = (int64_t)a.nq_pad * part.P;  // lists of the pass (the slots' stride)
  if (a.filter == FILTER_I8)
    hipLaunchKernelGGL((x1_replay_kernel<8, FILTER_I8>), grid, dim3(256), 0, st, a.dcount, a.dslot,
                       part.key, part.id, part.P, part.KP, a.nqa, a.qs, a.xs, a.self0, a.ntotal,
                       a.dR, nl, a.qcut, stats);
  else
    hipLaunchKernelGGL((x1_replay_kernel<8, FILTER_BF16>), grid, dim3(256), 0, st, a.dcount,
                       a.dslot, part.key, part.id, part.P, part.KP, a.nqa, a.qs, a.xs, a.self0,
                       a.ntotal, a.dR, nl, a.qcut, stats);
  return hipGetLastError();
}

// Filter-pass candidate count: the merged approximate candidates for `need`
// exact entries, with a margin of at least 8 (0 = not served by the filter).
int x1_list_len(int need) {
  return need + 8 <= 24   ? 24
         : need + 8 <= 32 ? 32
         : need + 8 <= 64 ? 64
         : need < 128 ? 128  // inner product k = 29 .. 64 (2k - 1 <= 127)
         : need < 256 ? 256  // inner product k = 65 .. 128, L2 k <= 255
         : need < 512 ? 512  // inner product k = 129 .. 256
         : need < kVerifyMaxKF ? kVerifyMaxKF  // inner product k = 257 .. 512, L2 k <= 1023
                               : 0;
}

// ---------------------------------------------------------------------------
// Per-index maxima for the bound: max |x|^2, max |x - hi(x)|^2 and
// max |x - hi(x)|^2 / |x|^2 over rows [0, n) (non-negative floats order as their
// bits; NaN sorts above every number and makes the bound non-finite).
__global__ __launch_bounds__(256) void bound_stats_kernel(const float* __restrict__ norms,
                                                          const float* __restrict__ rn2, int64_t n,
                                                          unsigned* __restrict__ out) {
  unsigned m0 = 0, m1 = 0, m2 = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float a = norms[i], r = rn2[i];
    m0 = max(m0, __float_as_uint(a) & 0x7FFFFFFFu);
    m1 = max(m1, __float_as_uint(r) & 0x7FFFFFFFu);
    if (a > 0.0f) m2 = max(m2, __float_as_uint(r / a) & 0x7FFFFFFFu);
    else if (r > 0.0f || a != a) m2 = 0x7F800000u;  // a residual without a norm: no bound
  }
  for (int o = 32; o > 0; o >>= 1) {
    m0 = max(m0, (unsigned)__shfl_xor((int)m0, o));
    m1 = max(m1, (unsigned)__shfl_xor((int)m1, o));
    m2 = max(m2, (unsigned)__shfl_xor((int)m2, o));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(out + 0, m0);
    atomicMax(out + 1, m1);
    atomicMax(out + 2, m2);
  }
}

hipError_t launch_bound_stats(const float* norms, const float* rn2, int64_t n, unsigned* out,
                              hipStream_t st, bool accumulate) {
  if (!accumulate) {
    hipError_t e = hipMemsetAsync(out, 0, 3 * sizeof(unsigned), st);
    if (e != hipSuccess) return e;
  }
  if (n <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(bound_stats_kernel, dim3((unsigned)blocks), dim3(256), 0, st, norms, rn2, n,
                     out);
  return hipGetLastError();
}

// |x - hi(x)|^2 of rows [r0, r0+n) (fp32 rows, stride ld), one wave per row,
// fp64 sums rounded up to float (an upper bound, as the verification needs).
__global__ __launch_bounds__(256) void resid_norms_kernel(const float* __restrict__ X, int64_t ld,
                                                          int64_t r0, int64_t n,
                                                          float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = X + (r0 + row) * ld;
  double s = 0.0;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = *(const f32x4*)(xr + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = v[i];
      const float hi = __uint_as_float((uint32_t)f32_to_bf16_rne(x) << 16);
      const double r = (double)x - (double)hi;
      s += r * r;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) {
    float f = (float)s;
    if ((double)f < s) f = nextafterf(f, INFINITY);
    out[r0 + row] = f;
  }
}

hipError_t launch_resid_norms(const float* X, int64_t ld, int64_t r0, int64_t n, float* out,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(resid_norms_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, ld,
                     r0, n, out);
  return hipGetLastError();
}

// int8 plane: code = rint(x / s), s = max|x| / 127 per row, clamped to +-127
// (a zero row has s = 0 and zero codes).  One wave per row: the row's maximum
// and finiteness, then the codes (4 per lane-store) and, when rn2 is given, the
// residual |x - s code|^2 in fp64 (s * code and x - s * code are exact there),
// rounded up to float; a non-finite row gets rn2 = +inf, which makes every
// bound non-finite (every query then goes to the exact engine).
template <typename RT>
__global__ __launch_bounds__(256) void quantize_i8_kernel(const RT* __restrict__ X, int64_t ld,
                                                          int64_t r0, int64_t n,
                                                          int8_t* __restrict__ codes,
                                                          float* __restrict__ scale,
                                                          float* __restrict__ rn2) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const RT* xr = X + (r0 + row) * ld;
  float m = 0.0f;
  bool bad = false;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = row4(xr + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bad |= !isfinite(v[i]);
      m = fmaxf(m, fabsf(v[i]));
    }
  }
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  bad = __any(bad);
  const float s = bad ? 0.0f : m / 127.0f;
  double acc = 0.0;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = row4(xr + c);
    uint32_t packed = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int code = 0;
      if (s > 0.0f) code = (int)fminf(fmaxf(rintf(v[i] / s), -127.0f), 127.0f);
      packed |= (uint32_t)(code & 0xFF) << (8 * i);
      const double r = (double)v[i] - (double)s * (double)code;
      acc += r * r;
    }
    *(uint32_t*)(codes + plane_offset(r0 + row, c, ld)) = packed;  // tile-major
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    scale[r0 + row] = s;
    if (rn2) {
      float f = (float)acc;
      if ((double)f < acc) f = nextafterf(f, INFINITY);
      rn2[r0 + row] = bad ? INFINITY : f;
    }
  }
}

// ---------------------------------------------------------------------------
// L2 on the int8 plane: the augmented inner product (vs_internal.h,
// launch_quantize_i8_l2aug).  faiss ranks an L2 index's rows by
// fl(fl(|q|^2 + n_x) - 2 fl(q.x)) (exhaustive_L2sqr_blas), i.e. by
// q.x - n_x / 2 up to rounding; with x' = [x, e_1 .. e_m], q' = [q, C .. C] and
// sum_j e_j = -n_x / (2 C), that is x'.q', an inner product the int8 filter
// pass runs unchanged (list and dump launches, cuts, replays).  After the pass
// the lane lists' keys A ~ n_x / 2 - q.x become L2 keys qn + 2A
// (launch_l2aug_map) and the verification runs in the L2 metric with the
// augmented bound (bound_key).  One wave per row; the codes are written four per
// lane-store, the extra block (m a multiple of 64) after the ld row columns.
__global__ __launch_bounds__(256) void quantize_i8_l2aug_kernel(
    const float* __restrict__ X, int64_t ld, int64_t r0, int64_t n, int64_t pld, int m, float C,
    float nref, const float* __restrict__ norms, int8_t* __restrict__ codes,
    float* __restrict__ scale, float* __restrict__ rn2, float* __restrict__ anorm) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = X + (r0 + row) * ld;
  float mx = 0.0f;
  bool bad = false;
  double sq = 0.0;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = *(const f32x4*)(xr + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bad |= !isfinite(v[i]);
      mx = fmaxf(mx, fabsf(v[i]));
      sq += (double)v[i] * (double)v[i];
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o));
    sq += __shfl_xor(sq, o);
  }
  bad = __any(bad);
  const bool rows = norms != nullptr;
  // the scale and the extra block's codes: rows an even split of T = rint(E / s)
  // (base + 1 on the first |rem| columns), queries c everywhere
  double E = 0.0;
  float s = 0.0f;
  int64_t T = 0;
  int cq = 0;
  if (rows) {
    E = ((double)nref - (double)norms[r0 + row]) / (2.0 * (double)C);
    bad |= !isfinite(E);
    const double sd = fmax((double)mx, fabs(E) / m) / 127.0;
    s = (float)sd;
    if ((double)s < sd) s = nextafterf(s, INFINITY);
    if (bad) s = 0.0f;
    if (s > 0.0f) {
      const double t = rint(E / (double)s);
      T = (int64_t)fmin(fmax(t, -127.0 * m), 127.0 * m);
    }
  } else {
    cq = mx > C ? max(1, min(127, (int)floorf(127.0f * (C / mx)))) : 127;
    s = bad ? 0.0f : C / (float)cq;
  }
  const int64_t base = T / m, rem = T - base * m;  // |rem| < m, the sign of T
  const int64_t sg = rem < 0 ? -1 : 1, nrem = rem < 0 ? -rem : rem;
  double acc = 0.0;
  for (int64_t c = lane * 4; c < pld; c += 256) {
    uint32_t packed = 0;
    if (c < ld) {
      const f32x4 v = *(const f32x4*)(xr + c);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int code = 0;
        if (s > 0.0f) code = (int)fminf(fmaxf(rintf(v[i] / s), -127.0f), 127.0f);
        packed |= (uint32_t)(code & 0xFF) << (8 * i);
        const double r = (double)v[i] - (double)s * (double)code;
        acc += r * r;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t j = c + i - ld;  // extra column j (0 .. m-1; pld = ld + m)
        int code = 0;
        if (j < m) {
          if (rows) {
            code = (int)(base + (j < nrem ? sg : 0));
          } else if (s > 0.0f) {
            code = cq;
            const double r = (double)C - (double)s * (double)cq;
            acc += r * r;
          }
        }
        packed |= (uint32_t)(code & 0xFF) << (8 * i);
      }
    }
    *(uint32_t*)(codes + plane_offset(r0 + row, c, pld)) = packed;  // tile-major
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) {
    scale[r0 + row] = s;
    auto up = [](double v) {
      float f = (float)v;
      if ((double)f < v) f = nextafterf(f, INFINITY);
      return f;
    };
    if (rows) {
      // the extra block: e_j = s c_j + delta, delta = (E - s T) / m (E's fp64
      // rounding folded into the margin); |e|^2 = s^2 sum c_j^2 + 2 delta s T + m delta^2
      const double dlt = fabs(E - (double)s * (double)T) + fabs(E) * 1e-15;
      const double d1 = (E - (double)s * (double)T) / m;
      const double cc = (double)(m - nrem) * (double)(base * base) +
                        (double)nrem * (double)((base + sg) * (base + sg));
      const double e2 = (double)s * (double)s * cc + 2.0 * d1 * (double)s * (double)T + m * d1 * d1;
      rn2[r0 + row] = bad ? INFINITY : up((acc + dlt * dlt / m) * (1.0 + 1e-12));
      if (anorm) anorm[r0 + row] = bad ? INFINITY : up((sq + fmax(e2, 0.0)) * (1.0 + 1e-12) + 1e-30);
    } else {
      rn2[r0 + row] = bad ? INFINITY : up(acc * (1.0 + 1e-12));
    }
  }
}

hipError_t launch_quantize_i8_l2aug(const float* X, int64_t ld, int64_t r0, int64_t n,
                                    const L2Aug& g, const float* norms, int8_t* codes,
                                    float* scale, float* rn2, float* anorm, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % 64 != 0 || g.m <= 0 || g.m % 64 != 0 || !(g.C > 0.0f) || !std::isfinite(g.nref) ||
      !rn2)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(quantize_i8_l2aug_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X,
                     ld, r0, n, ld + g.m, g.m, g.C, g.nref, norms, codes, scale, rn2, anorm);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void bf16_plane_l2aug_kernel(
    const float* __restrict__ X, int64_t ld, int64_t r0, int64_t n, float Cb, float nref,
    const float* __restrict__ norms, uint16_t* __restrict__ plane, float* __restrict__ rn2,
    float* __restrict__ anorm) {
  constexpr int m = kAugBf16;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = X + (r0 + row) * ld;
  const int64_t pld = ld + m;
  char* base = (char*)plane;
  const bool rows = norms != nullptr;
  const double E = rows ? ((double)nref - (double)norms[r0 + row]) / (2.0 * (double)Cb) : 0.0;
  const uint16_t eb = rows ? f32_to_bf16_rne((float)(E / m)) : f32_to_bf16_rne(Cb);
  const double es = (double)__uint_as_float((uint32_t)eb << 16);  // a stored extra entry
  double acc = 0.0, sq = 0.0;
  bool bad = !isfinite(E);
  for (int64_t c = lane * 4; c < pld; c += 256) {
    uint32_t lo, hi;
    if (c < ld) {
      const f32x4 v = *(const f32x4*)(xr + c);
      uint16_t b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        b[i] = f32_to_bf16_rne(v[i]);
        bad |= !isfinite(v[i]);
        const double h = (double)__uint_as_float((uint32_t)b[i] << 16);
        const double r = (double)v[i] - h;
        acc += r * r;
        sq += (double)v[i] * (double)v[i];
      }
      lo = (uint32_t)b[0] | ((uint32_t)b[1] << 16);
      hi = (uint32_t)b[2] | ((uint32_t)b[3] << 16);
    } else {  // the extra block (pld = ld + m)
      lo = (uint32_t)eb | ((uint32_t)eb << 16);
      hi = lo;
    }
    *(uint2*)(base + plane_offset(r0 + row, 2 * c, 2 * pld)) = make_uint2(lo, hi);
  }
  for (int o = 32; o > 0; o >>= 1) {
    acc += __shfl_xor(acc, o);
    sq += __shfl_xor(sq, o);
  }
  bad = __any(bad);
  if (lane == 0 && rows) {
    auto up = [](double v) {
      float f = (float)v;
      if ((double)f < v) f = nextafterf(f, INFINITY);
      return f;
    };
    // e_j = es + delta, delta = (E - m es) / m: the extra block's residual is
    // m delta^2 (E's fp64 rounding in the margin)
    const double d1 = (E - m * es) / m;
    const double dlt = fabs(d1) + fabs(E) * 1e-15 / m;
    rn2[r0 + row] = bad ? INFINITY : up((acc + m * dlt * dlt) * (1.0 + 1e-12));
    anorm[r0 + row] = bad ? INFINITY : up((sq + m * (es + d1) * (es + d1)) * (1.0 + 1e-12) + 1e-30);
  }
}

hipError_t launch_bf16_plane_l2aug(const float* X, int64_t ld, int64_t r0, int64_t n,
                                   const L2Aug& g, const float* norms, uint16_t* plane, float* rn2,
                                   float* anorm, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % 64 != 0 || !(g.Cb > 0.0f) || !std::isfinite(g.nref) || (norms && (!rn2 || !anorm)))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(bf16_plane_l2aug_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X,
                     ld, r0, n, g.Cb, g.nref, norms, plane, rn2, anorm);
  return hipGetLastError();
}

// The augmentation's statistics, two passes over the first rows: nref < 0:
// acc[0] += max|x| over the nonzero rows, acc[1] += their count, acc[2] = the
// largest norm; nref >= 0: acc[3] = max |nref - n_x| / max|x| (bits of a
// non-negative double order as its unsigned image).  One wave per row, one
// atomic set per block.
__global__ __launch_bounds__(256) void l2aug_stats_kernel(const float* __restrict__ X, int64_t ld,
                                                          int64_t r0, int64_t n,
                                                          const float* __restrict__ norms,
                                                          float nref, double* __restrict__ acc) {
  __shared__ double part[4][3];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * 4 + wv;
  float mx = 0.0f;
  if (row < n) {
    const float* xr = X + (r0 + row) * ld;
    for (int64_t c = lane * 4; c < ld; c += 256) {
      const f32x4 v = *(const f32x4*)(xr + c);
      mx = fmaxf(fmaxf(fmaxf(mx, fabsf(v[0])), fmaxf(fabsf(v[1]), fabsf(v[2]))), fabsf(v[3]));
    }
  }
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if (lane == 0) {
    const bool on = row < n && mx > 0.0f && isfinite(mx);
    const double nx = on ? (double)norms[r0 + row] : 0.0;
    part[wv][0] = on ? (double)mx : 0.0;
    part[wv][1] = on ? 1.0 : 0.0;
    const double r = nref < 0.0f ? nx : fabs((double)nref - nx) / (double)mx;
    part[wv][2] = on && isfinite(r) ? r : 0.0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0, c = 0.0;
    for (int i = 0; i < 4; ++i) {
      a += part[i][0];
      b += part[i][1];
      c = fmax(c, part[i][2]);
    }
    if (b > 0.0) {
      if (nref < 0.0f) {
        atomicAdd(acc + 0, a);
        atomicAdd(acc + 1, b);
      }
      atomicMax((unsigned long long*)(acc + (nref < 0.0f ? 2 : 3)),
                (unsigned long long)__double_as_longlong(c));
    }
  }
}

hipError_t l2aug_params(const float* X, int64_t ld, int64_t r0, int64_t n, const float* norms,
                        L2Aug* out, hipStream_t st) {
  out->m = 64;
  out->C = 1.0f;
  out->nref = 0.0f;
  out->Cb = 1.0f;
  if (n <= 0) return hipSuccess;
  double* acc = nullptr;
  hipError_t e = hipMalloc(&acc, 4 * sizeof(double));
  if (e != hipSuccess) return e;
  double h[4] = {0.0, 0.0, 0.0, 0.0};
  const dim3 grid((unsigned)((n + 3) / 4));
  e = hipMemsetAsync(acc, 0, 4 * sizeof(double), st);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(l2aug_stats_kernel, grid, dim3(256), 0, st, X, ld, r0, n, norms, -1.0f, acc);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  const float nref = (float)h[2];
  if (e == hipSuccess && h[1] > 0.0 && h[0] > 0.0 && std::isfinite(nref)) {
    hipLaunchKernelGGL(l2aug_stats_kernel, grid, dim3(256), 0, st, X, ld, r0, n, norms, nref, acc);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h, acc, sizeof(h), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) {
      const double c = h[0] / h[1];
      // a row's extra entries stay within its own max|x| when
      // m >= |nref - n_x| / (2 C max|x|)
      const double need = h[3] / (2.0 * c);
      out->C = (float)c;
      out->nref = nref;
      out->Cb = std::ldexp(1.0f, (int)std::lround(std::log2(c)));
      // capped at ld / 8 (at least 64 columns): a few tiny-but-nonzero rows
      // would otherwise widen every row of the plane (up to 4096 columns);
      // past the cap a row's extra entries exceed its max|x| and only its own
      // scale coarsens (quantize_i8_l2aug_kernel: s = max(max|x|, |E| / m) / 127)
      const double cap = std::max(64.0, std::ceil((double)ld / 8.0 / 64.0) * 64.0);
      out->m = (int)std::min<double>(cap, std::max(64.0, std::ceil(need / 64.0) * 64.0));
    }
  }
  (void)hipFree(acc);
  return e;
}

__global__ __launch_bounds__(256) void l2aug_map_kernel(float* __restrict__ key,
                                                        const int* __restrict__ id,
                                                        int64_t per_query, int nq,
                                                        const float* __restrict__ qn, float nref,
                                                        float* __restrict__ qcut) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (int64_t)nq * per_query && id[i] >= 0) {
    const float v = (qn[i / per_query] + nref) + 2.0f * key[i];
    key[i] = v < 0.0f ? 0.0f : v;
  }
  if (qcut && i < nq) {
    const float c = qcut[i];
    if (c < FLT_MAX && c > -FLT_MAX) {
      const float v = (qn[i] + nref) + 2.0f * c;
      qcut[i] = v < 0.0f ? 0.0f : v;
    }
  }
}

hipError_t launch_l2aug_map(float* key, const int* id, int64_t per_query, int nq, const float* qn,
                            float nref, float* qcut, hipStream_t st) {
  const int64_t tot = std::max<int64_t>((int64_t)nq * per_query, nq);
  if (tot <= 0) return hipSuccess;
  hipLaunchKernelGGL(l2aug_map_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, st, key, id,
                     per_query, nq, qn, nref, qcut);
  return hipGetLastError();
}

// Gathered batch of a later filter stage: slot s < *count takes query gl[s]
// (its fp32 row of `src`, stride ld, and its aux value; self row self0 + gl[s]
// when self0 >= 0); slots past the count are zero rows (aux 0, no self row).
// One wave per slot.
__global__ __launch_bounds__(256) void gather_queries_kernel(
    const float* __restrict__ src, int64_t ld, const float* __restrict__ aux,
    const int* __restrict__ gl, const int* __restrict__ count, int nslot, int64_t self0,
    float* __restrict__ dst, float* __restrict__ daux, int* __restrict__ drow) {
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= nslot) return;
  const bool on = s < *count;
  const int q = on ? gl[s] : 0;
  const f32x4* in = (const f32x4*)(src + (int64_t)q * ld);
  f32x4* out = (f32x4*)(dst + (int64_t)s * ld);
  for (int64_t c = lane; c < ld / 4; c += 64) out[c] = on ? in[c] : f32x4{0.f, 0.f, 0.f, 0.f};
  if (lane == 0) {
    if (daux) daux[s] = on && aux ? aux[q] : 0.0f;
    if (drow) drow[s] = on && self0 >= 0 ? (int)(self0 + q) : -1;
  }
}

hipError_t launch_gather_queries(const float* src, int64_t ld, const float* aux, const int* gl,
                                 const int* count, int nslot, int64_t self0, float* dst,
                                 float* daux, int* drow, hipStream_t st) {
  if (nslot <= 0) return hipSuccess;
  if (ld % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gather_queries_kernel, dim3((unsigned)((nslot + 3) / 4)), dim3(256), 0, st,
                     src, ld, aux, gl, count, nslot, self0, dst, daux, drow);
  return hipGetLastError();
}

// out[j] = outer[inner[j]] for j < *count (query ids of a gathered batch's
// flagged slots), one thread per slot of a fixed grid.
__global__ __launch_bounds__(256) void compose_list_kernel(const int* __restrict__ outer,
                                                           const int* __restrict__ inner,
                                                           const int* __restrict__ count, int n,
                                                           int* __restrict__ out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < n && j < *count) out[j] = outer[inner[j]];
}

hipError_t launch_compose_list(const int* outer, const int* inner, const int* count, int n,
                               int* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(compose_list_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     outer, inner, count, n, out);
  return hipGetLastError();
}

__global__ void window_count_kernel(const int* __restrict__ count, int w0, int cap,
                                    int* __restrict__ out) {
  const int c = *count - w0;
  *out = c < 0 ? 0 : (c > cap ? cap : c);
}

hipError_t launch_window_count(const int* count, int w0, int cap, int* out, hipStream_t st) {
  hipLaunchKernelGGL(window_count_kernel, dim3(1), dim3(1), 0, st, count, w0, cap, out);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void mul_arrays_kernel(const float* __restrict__ a,
                                                         const float* __restrict__ b, int64_t n,
                                                         float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

// out[2 g + b] = max of f[r] over the rows r of 32-row group g with bit 2 of r
// equal to b (f >= 0); n a multiple of 32.  outmin (optional): the minimum
// over the rows below nvalid (FLT_MAX for a part with none: padding rows,
// whose zero factors would otherwise make every dump launch's minimum 0).
__global__ __launch_bounds__(256) void group_max_kernel(const float* __restrict__ f, int64_t ngrp,
                                                        int64_t nvalid, float* __restrict__ out,
                                                        float* __restrict__ outmin) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (group, bit)
  if (i >= 2 * ngrp) return;
  const int64_t r0 = (i >> 1) * 32 + (i & 1) * 4;
  const float* p = f + r0;
  float m = 0.0f, mn = FLT_MAX;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 v = *(const f32x4*)(p + 8 * j);
    m = fmaxf(fmaxf(fmaxf(m, v[0]), fmaxf(v[1], v[2])), v[3]);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (r0 + 8 * j + e < nvalid) mn = fminf(mn, v[e]);
  }
  out[i] = m;
  if (outmin) outmin[i] = mn;
}

hipError_t launch_group_max(const float* f, int64_t n, float* out, hipStream_t st, int64_t nvalid,
                            float* outmin) {
  if (n <= 0) return hipSuccess;
  if (n % 32 != 0) return hipErrorInvalidValue;
  const int64_t m = 2 * (n / 32);
  hipLaunchKernelGGL(group_max_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, f,
                     n / 32, nvalid, out, outmin);
  return hipGetLastError();
}

hipError_t launch_mul_arrays(const float* a, const float* b, int64_t n, float* out,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(mul_arrays_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b,
                     n, out);
  return hipGetLastError();
}

hipError_t launch_quantize_i8(const void* X, int64_t ld, int64_t r0, int64_t n, int8_t* codes,
                              float* scale, float* rn2, hipStream_t st, int xesize) {
  if (n <= 0) return hipSuccess;
  if (ld % 4 != 0 || (xesize != 4 && xesize != 2)) return hipErrorInvalidValue;
  if (xesize == 4)
    hipLaunchKernelGGL(quantize_i8_kernel<float>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st,
                       (const float*)X, ld, r0, n, codes, scale, rn2);
  else
    hipLaunchKernelGGL(quantize_i8_kernel<uint16_t>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0,
                       st, (const uint16_t*)X, ld, r0, n, codes, scale, rn2);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Verification (engines VS_ENGINE_I8_VERIFY / VS_ENGINE_BF16_VERIFY).  Written
// for the bf16 plane; the int8 plane is the same argument with hi(.) the
// dequantized row s * code and gam its three scaling roundings (the int32 sum is
// exact), see make_bound_args.  With x = hi(x) + r(x) and
// q = hi(q) + r(q) (bf16 round-to-nearest-even, residuals exact in fp32):
//   x.q - hi(x).hi(q) = hi(x).r(q) + r(x).hi(q) + r(x).r(q)
// and the MFMA sums ld exact products in fp32 (each add off by <= 1 ulp), so
// for every row (Cauchy-Schwarz on each term)
//   |approx - x.q| <= gam |hi(x)||hi(q)| + |hi(x)||r(q)| + |r(x)||hi(q)| + |r(x)||r(q)|,
// gam = n u / (1 - n u), n = ld + 1, u = 2^-23; the exact key is the fp32
// rounding of x.q (one more 2^-23 |x||q|).  |hi(x)| <= |x| + |r(x)|, and the
// verification takes the maxima of |x| and |r(x)| over the index.  Let a = the
// sorted approximate keys of the KF candidates of a query and E their exact
// keys, sorted; E[M-1] bounds the true M-th best key from above, and every row
// outside the candidates has approximate key >= T (the KF-th candidate, or a
// full lane list's last entry, whichever is smaller), so whenever
//     T - B > E[M-1]
// the exact top-M (ties included) is among the candidates and E's first M
// entries are it.  Otherwise the query is flagged for the exact engine.


__device__ __forceinline__ double bound_key(int mode, const BoundArgs& ba, double qh2, double qr2,
                                            double qn2, const unsigned* stats) {
  if (ba.l2aug) {
    // L2 through the augmented int8 plane: stats are the maxima of |x'|^2 and
    // |x' - plane(x')|^2, qh2 / qr2 the query's |plane(q')|^2 bound and
    // |q' - plane(q')|^2, qn2 = |q|^2 as staged.  The pass's key A differs from
    // n_x / 2 - q.x by at most the inner-product bound b of the augmented
    // vectors (no fp32 key rounding inside: A is not rounded again); the list
    // key is max(0, fl(fl(qn + nref) + 2A)) (two more roundings, at most
    // 2u (qn + nref + 2 |A|)) and
    // the exact key fl(fl(qn + n_x) - fl(2 fl(q.x))) is within 8u (qn + n_x) of
    // qn + n_x - 2 q.x (as for the other L2 passes); max(0, .) is 1-Lipschitz.
    const double ax2 = (double)__uint_as_float(stats[0]);  // >= max |x|^2 too
    const double hx = sqrt(ax2) + sqrt((double)__uint_as_float(stats[1]));
    const double rx = sqrt((double)__uint_as_float(stats[1]));
    const double hq = sqrt(qh2), rq = sqrt(qr2);
    const double u = ldexp(1.0, -24);
    double b = ba.gam * hx * hq + hx * rq + rx * hq + rx * rq;
    b *= 1.0 + 1e-6;
    double B = 2.0 * b + 8.0 * u * (qn2 + ax2) + 2.0 * u * (qn2 + ba.aug_nref + 2.01 * hx * hq);
    // MODE_L2D (faiss's sequential formula, keys the rounded exact sum of
    // (x - q)^2): the pass's keys follow the stored fp32 norms, each within
    // norm_inf / 2 (relative) of the exact one, and the key's own rounding
    if (mode == MODE_L2D) B += (ba.norm_inf + 4.0 * u) * (qn2 + ax2);
    return B * (1.0 + 1e-6);
  }
  const double xm = sqrt((double)__uint_as_float(stats[0]) * (1.0 + ba.norm_inf));
  const double rx = ba.rows_exact ? 0.0 : sqrt((double)__uint_as_float(stats[1]));
  const double hx = xm + rx;
  const double hq = sqrt(qh2), rq = sqrt(qr2), qn = sqrt(qn2);
  double b = ba.gam * hx * hq + hx * rq + rx * hq + rx * rq + 2.0 * ldexp(1.0, -24) * xm * qn;
  b *= 1.0 + 1e-6;
  if (mode == MODE_L2 || mode == MODE_L2D) {  // key = (|q|^2 + |x|^2) - 2 ip, every step rounded
    const double xm2 = (double)__uint_as_float(stats[0]);
    b = 2.0 * b + 8.0 * ldexp(1.0, -24) * (qn2 + xm2);
    if (mode == MODE_L2D) b += (ba.norm_inf + 4.0 * ldexp(1.0, -24)) * (qn2 + xm2);
  } else if (mode == MODE_COS) {
    // keys -(s qinv xinv) with qinv, xinv from the stored norms (relative error
    // ~gam(ld) each, 1.5 norm_inf together); |s_a - s_e| / (|x||q|) <=
    // gam (1+rho)^2 + 2 rho (1+rho) + rho^2 + 2^-23, rho = max |r(x)| / |x| (the queries are stored rows); two roundings
    // of a key of magnitude <= 1 add 2^-22
    const double rho =
        ba.rows_exact ? 0.0 : sqrt((double)__uint_as_float(stats[2]) * (1.0 + ba.norm_inf));
    const double rel = ba.gam * (1 + rho) * (1 + rho) + 2 * rho * (1 + rho) + rho * rho +
                       ldexp(1.0, -23);
    b = (rel * (1.0 + 1.5 * ba.norm_inf) + ldexp(1.0, -22)) * (1.0 + 1e-6);
  }
  return b;
}

// the query's split norms |hi(q)|^2, |r(q)|^2, |q|^2 (fp64, across the wave);
// int8 plane (qr2i8 = the query's stored residual norm, rounded up):
// |hi(q)| <= |q| + |r(q)|
__device__ __forceinline__ void query_split_norms(const float* __restrict__ qrow, int64_t ld,
                                                  int lane, const float* __restrict__ qr2i8,
                                                  double& qh2, double& qr2, double& qn2,
                                                  double aug = 0.0) {
  double a = 0.0, r = 0.0, n = 0.0;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = *(const f32x4*)(qrow + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = v[i];
      const float hi = __uint_as_float((uint32_t)f32_to_bf16_rne(x) << 16);
      const double rr = (double)x - (double)hi;
      a += (double)hi * hi;
      r += rr * rr;
      n += (double)x * x;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    r += __shfl_xor(r, o);
    n += __shfl_xor(n, o);
  }
  qh2 = a + aug;  // aug: |q'|^2 = |q|^2 + m C^2 (the augmented L2 planes; exact
  qr2 = r;        // in bf16, whose extra entries are a power of two)
  qn2 = n;
  if (qr2i8) {
    qr2 = (double)*qr2i8;
    const double hq = sqrt(n + aug) + sqrt(qr2);
    qh2 = hq * hq;
  }
}

// exact dot product of two fp32 rows (fp64 accumulation across the wave);
// DIFF: the exact sum of (x - q)^2 instead (faiss's sequential L2 formula,
// MODE_L2D: each difference of two floats is exact in fp64, its square too)
template <bool DIFF = false, typename RT = float>
__device__ __forceinline__ double wave_dot(const RT* __restrict__ x, const float* __restrict__ q,
                                           int64_t ld, int lane) {
  double acc = 0.0;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 xv = row4(x + c);
    const f32x4 qv = *(const f32x4*)(q + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr (DIFF) {
        const double t = (double)xv[e] - (double)qv[e];
        acc = fma(t, t, acc);
      } else {
        acc = fma((double)xv[e], (double)qv[e], acc);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  return acc;
}

// The same sums for two rows at once against a query whose slice of this lane
// sits in registers (ld <= 256 kQV): every load of both rows is issued before
// the first FMA (one memory round trip per pair instead of one per 1 KB), and
// each row's terms are added in wave_dot's order (identical results).  (Four
// rows per step: the first check 51 vs 54 us at C2, the wide check 194 vs 130
// us at one wave per SIMD, profiles/r06tl2: both are bound by the rows' HBM
// gathers, ~3-4 TB/s.)
constexpr int kQV = 8;
struct QSlice {
  f32x4 v[kQV];
};
__device__ __forceinline__ void load_qslice(const float* __restrict__ q, int64_t ld, int lane,
                                            QSlice& qs) {
#pragma unroll
  for (int i = 0; i < kQV; ++i) {
    const int64_t c = lane * 4 + 256 * i;
    qs.v[i] = c < ld ? *(const f32x4*)(q + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}
template <bool DIFF = false, typename RT = float>
__device__ __forceinline__ void wave_dot2(const RT* __restrict__ xa, const RT* __restrict__ xb,
                                          const QSlice& qs, int64_t ld, int lane, double& ra,
                                          double& rb) {
  f32x4 va[kQV], vb[kQV];
#pragma unroll
  for (int i = 0; i < kQV; ++i) {
    const int64_t c = lane * 4 + 256 * i;
    va[i] = c < ld ? row4(xa + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    vb[i] = c < ld ? row4(xb + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int i = 0; i < kQV; ++i) {
    if (lane * 4 + 256 * i >= ld) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if constexpr (DIFF) {
        const double ta = (double)va[i][e] - (double)qs.v[i][e];
        const double tb = (double)vb[i][e] - (double)qs.v[i][e];
        a = fma(ta, ta, a);
        b = fma(tb, tb, b);
      } else {
        a = fma((double)va[i][e], (double)qs.v[i][e], a);
        b = fma((double)vb[i][e], (double)qs.v[i][e], b);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
  }
  ra = a;
  rb = b;
}

template <int MODE>
__device__ __forceinline__ float exact_key(float ip, int q, int r, const float* __restrict__ qn,
                                           const float* __restrict__ xn,
                                           const float* __restrict__ qinv,
                                           const float* __restrict__ xinv) {
  return MODE == MODE_L2    ? l2_from_ip(qn[q], xn[r], ip)
         : MODE == MODE_COS ? -(ip * (qinv[q] * xinv[r]))
         : MODE == MODE_L2D ? ip  // the rounded exact sum of (x - q)^2
                            : -ip;
}

// One wave per query.  Dk/Ik: the KF best approximate keys (ascending) and
// local rows; X/xn: fp32 rows (stride ld) and squared norms; Q: query rows
// (stride ld); qn: |q|^2 as staged for L2.  Writes KF exact (key, row) entries
// sorted, padded to KP, and fail[q].  NE = candidates per lane (KF <= 64 NE).
template <int MODE, int NE, typename RT>
__global__ __launch_bounds__(64) void verify_rescore_kernel(
    int KF, int M, const float* __restrict__ Dk, const int64_t* __restrict__ Ik,
    const RT* __restrict__ X, const float* __restrict__ xn, const float* __restrict__ Q,
    const float* __restrict__ qn, int64_t ld, BoundArgs ba, const unsigned* __restrict__ stats,
    const float* __restrict__ lkey, const int* __restrict__ lid, int P, int LKP, int L,
    float* __restrict__ okey, int* __restrict__ oid, int KP, int* __restrict__ fail,
    const float* __restrict__ qinv, const float* __restrict__ xinv, const float* __restrict__ qr2i8,
    const int* __restrict__ qcount, const float* __restrict__ qcut) {
  __shared__ float ek[64 * NE];
  __shared__ int sid[64 * NE];
  __shared__ float eMs;
  const int lane = threadIdx.x;
  const int q = blockIdx.x;
  if (qcount && q >= *qcount) {  // gathered batch: slots past the count are not flagged
    if (lane == 0) fail[q] = 0;
    return;
  }
  int id[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int j = lane + 64 * e;
    id[e] = j < KF ? (int)Ik[(int64_t)q * KF + j] : -1;
    sid[j] = id[e];
  }
  if (lane == 0) eMs = FLT_MAX;
  const float aK = Dk[(int64_t)q * KF + KF - 1];
  const int idK = (int)Ik[(int64_t)q * KF + KF - 1];
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
  if (qcut && qcut[q] < FLT_MAX) {  // the pass dropped every row at or above the cut
    bounded = true;
    T = fminf(T, qcut[q]);
  }

  const float* qrow = Q + (int64_t)q * ld;
  double qh2, qr2, qn2;
  query_split_norms(qrow, ld, lane, qr2i8 ? qr2i8 + q : nullptr, qh2, qr2, qn2, ba.aug_q2);
  if (ba.rows_exact) {  // the fp32 GEMM multiplied q itself
    qh2 = qn2;
    qr2 = 0.0;
  }
  __syncthreads();  // sid
  if (ld <= 256 * kQV) {  // two candidates per step, the query in registers
    QSlice qsl;
    load_qslice(qrow, ld, lane, qsl);
    for (int j = 0; j < KF; j += 2) {
      const int ra = sid[j], rb = j + 1 < KF ? sid[j + 1] : -1;
      double da, db;
      wave_dot2<MODE == MODE_L2D, RT>(X + (int64_t)max(ra, 0) * ld, X + (int64_t)max(rb, 0) * ld,
                                      qsl, ld, lane, da, db);
      if (lane == 0) {
        ek[j] = ra < 0 ? FLT_MAX : exact_key<MODE>((float)da, q, ra, qn, xn, qinv, xinv);
        if (j + 1 < KF) ek[j + 1] = rb < 0 ? FLT_MAX : exact_key<MODE>((float)db, q, rb, qn, xn, qinv, xinv);
      }
    }
  } else {
    for (int j = 0; j < KF; ++j) {
      const int r = sid[j];
      if (r < 0) {
        if (lane == 0) ek[j] = FLT_MAX;
        continue;
      }
      const double acc = wave_dot<MODE == MODE_L2D, RT>(X + (int64_t)r * ld, qrow, ld, lane);
      if (lane == 0) ek[j] = exact_key<MODE>((float)acc, q, r, qn, xn, qinv, xinv);
    }
  }
  __syncthreads();
  // rank sort of (key, row); empty slots last, in slot order among themselves
  float* ok = okey + (int64_t)q * KP;
  int* oi = oid + (int64_t)q * KP;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const int s = lane + 64 * e;
    if (s < KF) {
      const float k0 = ek[s];
      const int i0 = id[e] < 0 ? INT_MAX : id[e];
      int rank = 0;
      for (int j = 0; j < KF; ++j) {
        const float kj = ek[j];
        const int ij = sid[j] < 0 ? INT_MAX : sid[j];
        rank += (lex_less(kj, ij, k0, i0) || (kj == k0 && ij == i0 && j < s)) ? 1 : 0;
      }
      ok[rank] = k0;
      oi[rank] = id[e];  // -1 for empty slots
      if (rank == M - 1) eMs = k0;  // the M-th exact key
    } else if (s < KP) {
      ok[s] = FLT_MAX;
      oi[s] = -1;
    }
  }
  __syncthreads();
  const float eM = eMs;
  const double bkey = bound_key(MODE, ba, qh2, qr2,
                                MODE == MODE_L2 || MODE == MODE_L2D ? (double)qn[q] : qn2, stats);
  const bool pass = !bounded || ((double)T - bkey > (double)eM && isfinite(T) && isfinite(eM) &&
                                  isfinite(bkey));
  if (lane == 0) fail[q] = pass ? 0 : 1;
}

hipError_t launch_verify_rescore(int mode, int nq, int KF, int M, const float* Dk,
                                 const int64_t* Ik, const void* X, const float* xn,
                                 const float* Q, const float* qn, int64_t ld, const BoundArgs& ba,
                                 const unsigned* stats, Partials lists, int L, float* okey,
                                 int* oid, int KP, int* fail, hipStream_t st, const float* qinv,
                                 const float* xinv, const float* qr2i8, const int* qcount,
                                 const float* qcut, int xesize) {
  if (KF > kVerifyMaxKF || KP > kVerifyMaxKF || KF > KP || M < 1 || M > KF || ld % 4 != 0 ||
      L < 1 || L > lists.KP || (xesize != 4 && xesize != 2))
    return hipErrorInvalidValue;
  if (nq <= 0) return hipSuccess;
#define VS_VERIFY_T(MD, NE, RT)                                                                    \
  hipLaunchKernelGGL((verify_rescore_kernel<MD, NE, RT>), dim3(nq), dim3(64), 0, st, KF, M, Dk, Ik, \
                     (const RT*)X, xn, Q, qn, ld, ba, stats, lists.key, lists.id, lists.P,         \
                     lists.KP, L, okey, oid, KP, fail, qinv, xinv, qr2i8, qcount, qcut)
#define VS_VERIFY(MD, NE)                  \
  do {                                     \
    if (xesize == 4)                       \
      VS_VERIFY_T(MD, NE, float);          \
    else                                   \
      VS_VERIFY_T(MD, NE, uint16_t);       \
  } while (0)
#define VS_VERIFY_NE(MD)   \
  do {                     \
    if (KF <= 64)          \
      VS_VERIFY(MD, 1);    \
    else if (KF <= 128)    \
      VS_VERIFY(MD, 2);    \
    else if (KF <= 256)    \
      VS_VERIFY(MD, 4);    \
    else if (KF <= 512)    \
      VS_VERIFY(MD, 8);    \
    else                   \
      VS_VERIFY(MD, 16);   \
  } while (0)
  if (mode == MODE_IP)
    VS_VERIFY_NE(MODE_IP);
  else if (mode == MODE_L2)
    VS_VERIFY_NE(MODE_L2);
  else if (mode == MODE_L2D)
    VS_VERIFY_NE(MODE_L2D);
  else if (mode == MODE_COS && qinv && xinv)
    VS_VERIFY_NE(MODE_COS);
  else
    return hipErrorInvalidValue;
#undef VS_VERIFY_NE
#undef VS_VERIFY
#undef VS_VERIFY_T
  return hipGetLastError();
}

// Flagged queries -> ascending list qlist[0 .. *count) (one workgroup; a
// block-wide prefix count per 1024-query chunk).  Running statistics: adds
// the count to *total and n to *total_n (when not null).
__global__ __launch_bounds__(1024) void compact_flags_kernel(const int* __restrict__ flags, int n,
                                                             int* __restrict__ list,
                                                             int* __restrict__ count,
                                                             unsigned long long* __restrict__ total,
                                                             unsigned long long* __restrict__ total_n) {
  __shared__ int wsum[16];
  __shared__ int base;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < n; c0 += 1024) {
    const int i = c0 + tid;
    const int f = i < n && flags[i] != 0 ? 1 : 0;
    const uint64_t bal = __ballot(f);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wv] = __popcll(bal);
    __syncthreads();
    int off = base;
    for (int j = 0; j < wv; ++j) off += wsum[j];
    if (f) list[off + before] = i;
    __syncthreads();
    if (tid == 0) {
      int s = 0;
      for (int j = 0; j < 16; ++j) s += wsum[j];
      base += s;
    }
    __syncthreads();
  }
  if (tid == 0) {
    *count = base;
    if (total) atomicAdd(total, (unsigned long long)base);
    if (total_n) atomicAdd(total_n, (unsigned long long)n);
  }
}

// acc[0] += n, acc[1] += *count (one thread; a per-index record of a stage)
__global__ void add_counts_kernel(const int* __restrict__ count, int n,
                                  unsigned long long* __restrict__ acc) {
  // atomic: searches of one index on two streams may run this concurrently
  atomicAdd(acc + 0, (unsigned long long)n);
  atomicAdd(acc + 1, (unsigned long long)*count);
}

hipError_t launch_add_counts(const int* count, int n, unsigned long long* acc, hipStream_t st) {
  hipLaunchKernelGGL(add_counts_kernel, dim3(1), dim3(1), 0, st, count, n, acc);
  return hipGetLastError();
}

hipError_t launch_compact_flags(const int* flags, int n, int* list, int* count,
                                unsigned long long* total, unsigned long long* total_n,
                                hipStream_t st) {
  if (n < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(compact_flags_kernel, dim3(1), dim3(1024), 0, st, flags, n, list, count,
                     total, total_n);
  return hipGetLastError();
}

// Wide verification of the flagged queries qlist[0 .. *count) (one 256-thread
// workgroup per flagged query, a fixed grid striding over the device-side
// count, so the host never reads it).  The condition above only needs a
// threshold T such that every row outside the rescored set has approximate key
// >= T: the smallest last entry of the full lane lists is one (a full list
// dropped only rows lexicographically after its last entry), and then the set
// may be *all* list entries below T, not just the KF merged ones.  More than
// kWideCap entries below T, fewer than M, or a non-finite key: the query stays
// flagged.  The KF merged candidates the first check rescored (Dk/Ik, exact
// keys in okey/oid) keep their exact keys: an entry lexicographically at or
// before the KF-th merged one is one of them, and only the others are read
// from HBM again (C4: ~40 % of the wide set).
template <int MODE, typename RT>
__global__ __launch_bounds__(256) void verify_wide_kernel(
    const int* __restrict__ qlist, const int* __restrict__ count, int KF, int M,
    const RT* __restrict__ X, const float* __restrict__ xn, const float* __restrict__ Q,
    const float* __restrict__ qn, int64_t ld, BoundArgs ba, const unsigned* __restrict__ stats,
    const float* __restrict__ lkey, const int* __restrict__ lid, int P, int LKP, int L,
    float* __restrict__ okey, int* __restrict__ oid, int KP, int* __restrict__ fail,
    const float* __restrict__ qinv, const float* __restrict__ xinv, const float* __restrict__ qr2i8,
    const float* __restrict__ Dk, const int64_t* __restrict__ Ik,
    unsigned long long* __restrict__ sizes, const float* __restrict__ qcut) {
  __shared__ float ck[kWideCap];
  __shared__ int cid[kWideCap];
  // the first check's exact keys (KP <= kVerifyMaxKF) / the reused ones
  __shared__ float rk[kVerifyMaxKF], kk[kVerifyMaxKF];
  __shared__ int ri[kVerifyMaxKF], ki[kVerifyMaxKF];
  __shared__ int cntk;
  __shared__ float wT[4];
  __shared__ int wB[4];
  __shared__ int cnt, bad;
  __shared__ float eMs;
  __shared__ double qs[3];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int nflag = *count;
  for (int jq = blockIdx.x; jq < nflag; jq += gridDim.x) {
    const int q = qlist[jq];
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
      cntk = 0;
      bad = 0;
      eMs = FLT_MAX;
    }
    for (int t = tid; t < kVerifyMaxKF; t += 256) {  // the first check's output (KP entries)
      rk[t] = t < KP ? okey[(int64_t)q * KP + t] : FLT_MAX;
      ri[t] = t < KP ? oid[(int64_t)q * KP + t] : -1;
    }
    const float* qrow = Q + (int64_t)q * ld;
    if (wv == 0) {
      double a, b, c;
      query_split_norms(qrow, ld, lane, qr2i8 ? qr2i8 + q : nullptr, a, b, c, ba.aug_q2);
      if (lane == 0) {
        qs[0] = a;
        qs[1] = b;
        qs[2] = c;
      }
    }
    __syncthreads();
    T = fminf(fminf(wT[0], wT[1]), fminf(wT[2], wT[3]));
    bounded = (wB[0] | wB[1] | wB[2] | wB[3]) != 0;
    if (qcut && qcut[q] < FLT_MAX) {  // the pass dropped every row at or above the cut
      bounded = true;
      T = fminf(T, qcut[q]);
    }
    const double bkey =
        bound_key(MODE, ba, qs[0], qs[1],
                  MODE == MODE_L2 || MODE == MODE_L2D ? (double)qn[q] : qs[2], stats);
    // Any threshold T' <= T works (every row outside the set still has an
    // approximate key >= T'): with a_M the M-th smallest approximate key (the
    // merge's Dk), the M best-approximate rows have exact keys <= a_M + B, so
    // T' = a_M + 2B passes the check whenever it is below T, and rescoring only
    // the entries below T' keeps the set small when the lists reach deep (many
    // lists per query: T far behind the top).
    // Tighter still: e1_M, the M-th exact key among the first check's KF rows,
    // bounds E_M from above, and every row with approximate key >= e1_M + B has
    // an exact key > e1_M >= E_M; those M rows (approximate keys <= e1_M + B)
    // stay in the set.  T' = e1_M + B is ~a_M + B: half the window of a_M + 2B.
    if (bounded && Dk) {
      const float aM = Dk[(int64_t)q * KF + M - 1];
      double tp = (double)aM + 2.000001 * bkey;
      if (ri[M - 1] >= 0 && isfinite(rk[M - 1]))
        tp = fmin(tp, (double)rk[M - 1] + 1.000001 * bkey);
      if (isfinite(tp) && tp < (double)T) {
        float t = (float)tp;
        if ((double)t < tp) t = nextafterf(t, INFINITY);
        T = fminf(T, t);
      }
    }
    // the KF-th merged entry: entries up to it were rescored by the first check
    // (all of them when the merge found fewer than KF)
    const float kfk = Dk ? Dk[(int64_t)q * KF + KF - 1] : -FLT_MAX;
    const int kfi = Dk ? (int)Ik[(int64_t)q * KF + KF - 1] : INT_MIN;
    // gather every entry below T (all entries when no list is full)
    for (int j = tid; j < P * L; j += 256) {
      const int64_t o = lbase + (int64_t)(j / L) * LKP + j % L;
      const int r = lid[o];
      const float lk = lkey[o];
      if (r >= 0 && (!bounded || lk < T)) {
        int hit = -1;
        if (Dk && (kfi < 0 || !lex_less(kfk, kfi, lk, r)))
          for (int t = 0; t < KP; ++t) hit = ri[t] == r ? t : hit;
        if (hit >= 0) {
          const int s = atomicAdd(&cntk, 1);
          if (s < kVerifyMaxKF) {
            kk[s] = rk[hit];
            ki[s] = r;
          }
        } else {
          const int s = atomicAdd(&cnt, 1);
          if (s < kWideCap) cid[s] = r;
        }
      }
    }
    __syncthreads();
    const int nu = cnt;  // rows to rescore
    const int nk = min(cntk, kVerifyMaxKF);
    const int n = nu + cntk;
    if (sizes && tid == 0) {
      atomicAdd(sizes, (unsigned long long)n);
      atomicAdd(sizes + 1, (unsigned long long)nu);
    }
    if (!(n > kWideCap || n < M || !isfinite(T))) {  // uniform
      auto put = [&](int j, int r, double acc) {
        if (lane == 0) {
          const float key = exact_key<MODE>((float)acc, q, r, qn, xn, qinv, xinv);
          ck[j] = key;
          if (!isfinite(key)) bad = 1;
        }
      };
      if (ld <= 256 * kQV) {  // two rows per wave step, the query in registers
        QSlice qsl;
        load_qslice(qrow, ld, lane, qsl);
        for (int j = wv; j < nu; j += 8) {
          const int ra = cid[j], rb = j + 4 < nu ? cid[j + 4] : ra;
          double da, db;
          wave_dot2<MODE == MODE_L2D, RT>(X + (int64_t)ra * ld, X + (int64_t)rb * ld, qsl, ld, lane, da,
                                      db);
          put(j, ra, da);
          if (j + 4 < nu) put(j + 4, rb, db);
        }
      } else {
        for (int j = wv; j < nu; j += 4) {
          const int r = cid[j];
          put(j, r, wave_dot<MODE == MODE_L2D, RT>(X + (int64_t)r * ld, qrow, ld, lane));
        }
      }
      for (int t = tid; t < nk; t += 256) {  // the reused exact keys after the rescored ones
        ck[nu + t] = kk[t];
        cid[nu + t] = ki[t];
        if (!isfinite(kk[t])) bad = 1;
      }
      __syncthreads();
      if (!bad) {  // uniform
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
        const bool pass =
            !bounded || ((double)T - bkey > (double)eM && isfinite(eM) && isfinite(bkey));
        if (tid == 0 && pass) fail[q] = 0;
      }
    }
    __syncthreads();  // the shared state is reused by the next flagged query
  }
}

hipError_t launch_verify_wide(int mode, int nq_max, const int* qlist, const int* count, int KF,
                              int M, const void* X, const float* xn, const float* Q,
                              const float* qn, int64_t ld, const BoundArgs& ba,
                              const unsigned* stats, Partials lists, int L, float* okey, int* oid,
                              int KP, int* fail, hipStream_t st, const float* qinv,
                              const float* xinv, const float* qr2i8, const float* Dk,
                              const int64_t* Ik, unsigned long long* sizes,
                              const float* qcut, int xesize) {
  if (KF > KP || KP > kVerifyMaxKF || (Dk && !Ik) || M < 1 || M > KF || ld % 4 != 0 || L < 1 ||
      L > lists.KP || (xesize != 4 && xesize != 2))
    return hipErrorInvalidValue;
  if (nq_max <= 0) return hipSuccess;
  const int grid = std::min(nq_max, 2048);
#define VS_WIDE_T(MD, RT)                                                                         \
  hipLaunchKernelGGL((verify_wide_kernel<MD, RT>), dim3(grid), dim3(256), 0, st, qlist, count, KF, \
                     M, (const RT*)X, xn, Q, qn, ld, ba, stats, lists.key, lists.id, lists.P,     \
                     lists.KP, L, okey, oid, KP, fail, qinv, xinv, qr2i8, Dk, Ik, sizes, qcut)
#define VS_WIDE(MD)             \
  do {                          \
    if (xesize == 4)            \
      VS_WIDE_T(MD, float);     \
    else                        \
      VS_WIDE_T(MD, uint16_t);  \
  } while (0)
  if (mode == MODE_IP)
    VS_WIDE(MODE_IP);
  else if (mode == MODE_L2)
    VS_WIDE(MODE_L2);
  else if (mode == MODE_L2D)
    VS_WIDE(MODE_L2D);
  else if (mode == MODE_COS && qinv && xinv)
    VS_WIDE(MODE_COS);
  else
    return hipErrorInvalidValue;
#undef VS_WIDE
#undef VS_WIDE_T
  return hipGetLastError();
}

// Bound constants for `ld` K elements (see above).  bf16: the MFMA's fp32
// accumulation.  int8: the int32 sum is exact (|code| <= 127, ld <= kI8MaxLd),
// and the approximate score fl(fl(float(sum)) * fl(f_q * f_x)) carries three
// roundings for IP (f = s), five for the cosine (f = fl(s * inverse norm)), so
// approx = hi(x).hi(q) (1 + d), |d| <= (1 + 2^-24)^5 - 1 < 6 * 2^-24; for the
// cosine the key then needs no further rounding term (the 2^-22 kept below is
// slack).
// ---------------------------------------------------------------------------
// Query cuts.  The verification (above) needs every row outside the rescored
// set to have an approximate key >= its threshold T, and only ever uses
// T' = min(T, a_M + 2.000001 B, ...) (wide check) or passes iff T - B > E_M with
// E_M <= a_M + B (first check).  Every row with approximate key >= a_M + 2 B
// is therefore useless to both, and a_M, the M-th smallest key over a query's
// lane lists, only falls while the pass runs.  After the first launch of a
// pass, x1_qcut sets cut[q] = min(cut[q], a_M(now) + 2.000001 B) (rounded up);
// the dump launches that follow keep only the blocks that may hold a row below
// the cut, x1_replay admits their rows against min(list last, cut), and the
// verification takes T = min(T, cut) as the floor of the rows dropped that way.
// Since the final a_M <= a_M(now), the cut is never below the verification's
// own a_M + 2B: no check changes its outcome, and the lists only lose rows that
// could never enter the rescored set.  What it saves: a lane list admits rows
// against its own 8th entry (the 8th best of a 1/128 slice of the corpus at C3);
// the cut is the M-th best over all of them plus 2B, so a dump launch finds a
// block below it only for ~1 in 40 (lane, block) pairs — rare enough that a
// wave almost never waits on one (tests/test_filter_argument.py models it).

// bkey[q]: the bound B of query q (bound_key over its split norms, the same
// double the verification computes).
template <int MODE>
__global__ __launch_bounds__(64) void qbound_kernel(const float* __restrict__ Q, int64_t ld,
                                                    const float* __restrict__ qn, BoundArgs ba,
                                                    const unsigned* __restrict__ stats,
                                                    const float* __restrict__ qr2i8, int nq,
                                                    double* __restrict__ bkey) {
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  if (q >= nq) return;
  double qh2, qr2, qn2;
  query_split_norms(Q + (int64_t)q * ld, ld, lane, qr2i8 ? qr2i8 + q : nullptr, qh2, qr2, qn2,
                    ba.aug_q2);
  double b = bound_key(MODE, ba, qh2, qr2,
                                MODE == MODE_L2 || MODE == MODE_L2D ? (double)qn[q] : qn2, stats);
  // the augmented L2 pass cuts its lists in the inner-product keys A, whose
  // map qn + 2A doubles distances: half the L2 bound there
  if (ba.l2aug) b *= 0.5;
  if (lane == 0) bkey[q] = b;
}

__device__ __forceinline__ uint32_t key_order(float f) {  // float order as unsigned order
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_unorder(uint32_t u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// The KF = 128 or 256 best approximate candidates of each query (KF <= 64 goes
// through merge_lists_kernel, whose register lists would not hold 128): one
// 256-thread workgroup per query finds the KF-th smallest 64-bit image
// (key order << 32 | row; a query's lists hold distinct rows) of its P lists of
// L entries by a radix select, keeps the entries at or below it and ranks
// them.  Writes Dk/Ik [nq][KF] ascending (FLT_MAX / -1 padding).
__global__ __launch_bounds__(256) void select_lists_kernel(const float* __restrict__ lkey,
                                                           const int* __restrict__ lid, int P,
                                                           int LKP, int L, int KF,
                                                           float* __restrict__ Dk,
                                                           int64_t* __restrict__ Ik,
                                                           const int* __restrict__ qcount) {
  __shared__ int wsum[4];
  __shared__ unsigned long long sel[kVerifyMaxKF];
  __shared__ int nsel;
  __shared__ int hist[256];
  __shared__ int sel_digit, sel_before;
  const int q = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (qcount && q >= *qcount) return;  // gathered batch: slots past the count
  const int64_t base = (int64_t)q * P * LKP;
  const int n = P * L;
  constexpr int kR = 16;
  constexpr unsigned long long kNone = ~0ull;
  unsigned long long v[kR];
  const bool regs = n <= 256 * kR;  // uniform
  auto image = [&](int j) -> unsigned long long {
    const int64_t o = base + (int64_t)(j / L) * LKP + j % L;
    const int r = lid[o];
    return r >= 0 ? ((unsigned long long)key_order(lkey[o]) << 32) | (uint32_t)r : kNone;
  };
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const int j = tid + 256 * i;
    v[i] = regs && j < n ? image(j) : kNone;
  }
  auto count_le = [&](unsigned long long y) {  // entries with image <= y (workgroup-wide)
    int c = 0;
    if (regs) {
#pragma unroll
      for (int i = 0; i < kR; ++i) c += v[i] <= y && v[i] != kNone ? 1 : 0;
    } else {
      for (int j = tid; j < n; j += 256) {
        const unsigned long long x = image(j);
        c += x <= y && x != kNone ? 1 : 0;
      }
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __syncthreads();
    if (lane == 0) wsum[wv] = c;
    __syncthreads();
    return wsum[0] + wsum[1] + wsum[2] + wsum[3];
  };
  const int total = count_le(kNone - 1);
  const int M = total < KF ? total : KF;
  // the M-th smallest image y, by a radix select over its eight bytes from the
  // top: per byte a 256-bin histogram of the entries that share the bytes
  // chosen so far, the bin where the running count reaches the rank left
  // (8 passes over the entries instead of a bitwise search's 64: one query's
  // select is one workgroup's latency, a batch-1 search waits for all of it)
  unsigned long long y = kNone - 1;
  if (M > 0 && M < total) {
    unsigned long long pre = 0;
    int want = M;  // rank of y among the entries that share pre's chosen bytes
    for (int sh = 56; sh >= 0; sh -= 8) {
      hist[tid] = 0;  // 256 threads, 256 bins
      __syncthreads();
      auto add = [&](unsigned long long x) {
        if (x != kNone && (sh == 56 || (x >> (sh + 8)) == (pre >> (sh + 8))))
          atomicAdd(&hist[(int)((x >> sh) & 0xFF)], 1);
      };
      if (regs) {
#pragma unroll
        for (int i = 0; i < kR; ++i) add(v[i]);
      } else {
        for (int j = tid; j < n; j += 256) add(image(j));
      }
      __syncthreads();
      if (wv == 0) {  // the bin where the running count reaches `want`
        const int h0 = hist[4 * lane], h1 = hist[4 * lane + 1], h2 = hist[4 * lane + 2],
                  h3 = hist[4 * lane + 3];
        const int own = h0 + h1 + h2 + h3;
        int inc = own;  // inclusive prefix over the lanes
        for (int o = 1; o < 64; o <<= 1) {
          const int t = __shfl_up(inc, o);
          if (lane >= o) inc += t;
        }
        const int before = inc - own;
        if (before < want && want <= inc) {
          int c = before, d = 4 * lane;
          const int hh[4] = {h0, h1, h2, h3};
          for (int e = 0; e < 4; ++e) {
            if (c + hh[e] >= want) {
              d = 4 * lane + e;
              break;
            }
            c += hh[e];
          }
          sel_digit = d;
          sel_before = c;
        }
      }
      __syncthreads();
      pre |= (unsigned long long)sel_digit << sh;
      want -= sel_before;
      __syncthreads();  // hist and the broadcast are rewritten by the next byte
    }
    y = pre;  // the entries are distinct: y is the M-th smallest image
  }
  if (tid == 0) nsel = 0;
  __syncthreads();
  auto take = [&](unsigned long long x) {
    if (x != kNone && x <= y) {
      const int s = atomicAdd(&nsel, 1);
      if (s < kVerifyMaxKF) sel[s] = x;
    }
  };
  if (M > 0) {
    if (regs) {
#pragma unroll
      for (int i = 0; i < kR; ++i) take(v[i]);
    } else {
      for (int j = tid; j < n; j += 256) take(image(j));
    }
  }
  __syncthreads();
  float* dk = Dk + (int64_t)q * KF;
  int64_t* ik = Ik + (int64_t)q * KF;
  for (int t = tid; t < KF; t += 256) {
    if (t < M) {
      const unsigned long long x = sel[t];
      int rank = 0;
      for (int j = 0; j < M; ++j) rank += sel[j] < x ? 1 : 0;
      dk[rank] = key_unorder((uint32_t)(x >> 32));
      ik[rank] = (int64_t)(uint32_t)(x & 0xFFFFFFFFull);
    } else {
      dk[t] = FLT_MAX;
      ik[t] = -1;
    }
  }
}

hipError_t launch_select_lists(Partials part, int L, int nq, int KF, float* Dk, int64_t* Ik,
                               hipStream_t st, const int* qcount) {
  if (KF < 1 || KF > kVerifyMaxKF || L < 1 || L > part.KP || part.P < 1) return hipErrorInvalidValue;
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(select_lists_kernel, dim3(nq), dim3(256), 0, st, part.key, part.id, part.P,
                     part.KP, L, KF, Dk, Ik, qcount);
  return hipGetLastError();
}

// The KF <= 64 best approximate candidates of each query from its P sorted
// lane lists of 8 entries (stride 8), by a bound from the lists' heads instead
// of merge_lists_kernel's six rounds of 32-entry merges (C2: 35-38 us vs the
// merge's 94 in two levels, profiles/r06tl2).  The KF-th smallest head U (lexicographic (key, row);
// a query's lists hold distinct rows) bounds the KF-th smallest entry: the KF
// lists of the smallest heads hold KF entries <= U.  Only those lists can hold
// an entry <= U, so at most 8 KF entries (<= 512) are kept and ranked.  Fewer
// than KF non-empty lists: every entry is kept.  Same output as the merge:
// Dk/Ik [nq][KF] ascending, (FLT_MAX, -1) padding.
constexpr int kHeadsMaxP = 512;
constexpr int kHeadsMaxKF = 64;
__global__ __launch_bounds__(256) void select_heads_kernel(const float* __restrict__ lkey,
                                                           const int* __restrict__ lid, int P,
                                                           int KF, float* __restrict__ Dk,
                                                           int64_t* __restrict__ Ik,
                                                           const int* __restrict__ qcount) {
  __shared__ float hk[kHeadsMaxP];
  __shared__ int hi[kHeadsMaxP];
  __shared__ float ck[8 * kHeadsMaxKF];
  __shared__ int ci[8 * kHeadsMaxKF];
  __shared__ int cnt, ui;
  __shared__ float uk;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  if (qcount && q >= *qcount) return;  // gathered batch: slots past the count
  const int64_t base = (int64_t)q * P * 8;
  for (int p = tid; p < P; p += 256) {
    hk[p] = lkey[base + (int64_t)p * 8];
    hi[p] = lid[base + (int64_t)p * 8];
  }
  if (tid == 0) {
    cnt = 0;
    ui = -1;  // no bound: fewer than KF non-empty lists
    uk = FLT_MAX;
  }
  __syncthreads();
  for (int p = tid; p < P; p += 256) {
    const float k0 = hk[p];
    const int i0 = hi[p];
    if (i0 < 0) continue;
    int r = 0;
    for (int t = 0; t < P; ++t) r += hi[t] >= 0 && lex_less(hk[t], hi[t], k0, i0) ? 1 : 0;
    if (r == KF - 1) {
      uk = k0;
      ui = i0;
    }
  }
  __syncthreads();
  const float U = uk;
  const int Ui = ui;
  for (int p = tid; p < P; p += 256) {
    if (Ui >= 0 && lex_less(U, Ui, hk[p], hi[p])) continue;  // head above the bound
    const f32x4* kp = (const f32x4*)(lkey + base + (int64_t)p * 8);
    const int4* ip = (const int4*)(lid + base + (int64_t)p * 8);
    const f32x4 ka = kp[0], kb = kp[1];
    const int4 ia = ip[0], ib = ip[1];
    const float kk[8] = {ka.x, ka.y, ka.z, ka.w, kb.x, kb.y, kb.z, kb.w};
    const int ii[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (ii[j] < 0 || (Ui >= 0 && lex_less(U, Ui, kk[j], ii[j]))) break;  // sorted: the rest too
      const int s = atomicAdd(&cnt, 1);
      if (s < 8 * kHeadsMaxKF) {
        ck[s] = kk[j];
        ci[s] = ii[j];
      }
    }
  }
  __syncthreads();
  // <= 8 KF: at most KF lists pass the head test when bounded
  const int n = min(cnt, 8 * kHeadsMaxKF);
  float* dk = Dk + (int64_t)q * KF;
  int64_t* ik = Ik + (int64_t)q * KF;
  for (int j = tid; j < n; j += 256) {
    const float k0 = ck[j];
    const int i0 = ci[j];
    int r = 0;
    for (int t = 0; t < n; ++t) r += lex_less(ck[t], ci[t], k0, i0) ? 1 : 0;
    if (r < KF) {
      dk[r] = k0;
      ik[r] = i0;
    }
  }
  for (int j = n + tid; j < KF; j += 256) {
    dk[j] = FLT_MAX;
    ik[j] = -1;
  }
}

bool select_heads_applies(const Partials& part, int L, int KF) {
  const char* e = getenv("VS_SELECT_HEADS");  // =0: the list merge (A/B; read at every search)
  if (e && atoi(e) == 0) return false;
  return L == 8 && part.KP == 8 && KF >= 1 && KF <= kHeadsMaxKF && part.P >= KF &&
         part.P <= kHeadsMaxP;
}

hipError_t launch_select_heads(Partials part, int nq, int KF, float* Dk, int64_t* Ik,
                               hipStream_t st, const int* qcount) {
  if (!select_heads_applies(part, 8, KF)) return hipErrorInvalidValue;
  if (nq <= 0) return hipSuccess;
  hipLaunchKernelGGL(select_heads_kernel, dim3(nq), dim3(256), 0, st, part.key, part.id, part.P,
                     KF, Dk, Ik, qcount);
  return hipGetLastError();
}

// One workgroup of 256 threads per query: a_M = the M-th smallest key over
// the query's P lists of L entries (bitwise search on the order-preserving
// integer image), then the cut.  Fewer than M entries: no cut yet.  Up to 4,096
// entries stay in registers (C2: 256 lists x 8; one wave re-reading 2,048
// entries from memory per count cost ~0.8 ms per search, profiles/r05l), more
// are read again per count.
constexpr int kQcutThreads = 256;
__global__ __launch_bounds__(kQcutThreads) void qcut_kernel(
    const float* __restrict__ lkey, const int* __restrict__ lid, int P, int LKP, int L, int M,
    const double* __restrict__ bkey, int nq, float* __restrict__ cut) {
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  if (q >= nq) return;  // uniform over the workgroup
  const int64_t base = (int64_t)q * P * LKP;
  const int n = P * L;
  // order images (uint64; empty entries 2^32, never counted)
  constexpr int kR = 16;
  uint64_t v[kR];
  const bool regs = n <= kQcutThreads * kR;  // uniform
  auto image = [&](int j) -> uint64_t {
    const int64_t o = base + (int64_t)(j / L) * LKP + j % L;
    return lid[o] >= 0 ? (uint64_t)key_order(lkey[o]) : (1ull << 32);
  };
#pragma unroll
  for (int i = 0; i < kR; ++i) {
    const int j = tid + kQcutThreads * i;
    v[i] = regs && j < n ? image(j) : (1ull << 32);
  }
  __shared__ int part[kQcutThreads / 64];
  auto count_below = [&](uint64_t y) {  // entries with order image < y (uniform result)
    int c = 0;
    if (regs) {
#pragma unroll
      for (int i = 0; i < kR; ++i) c += v[i] < y ? 1 : 0;
    } else {
      for (int j = tid; j < n; j += kQcutThreads) c += image(j) < y ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __syncthreads();  // the previous count's reads of part[] are done
    if ((tid & 63) == 0) part[tid >> 6] = c;
    __syncthreads();
    int t = 0;
#pragma unroll
    for (int w = 0; w < kQcutThreads / 64; ++w) t += part[w];
    return t;
  };
  if (count_below(1ull << 32) < M) return;  // uniform
  // the largest x with fewer than M entries below it: the M-th smallest image
  uint64_t x = 0;
  for (int b = 31; b >= 0; --b)
    if (count_below(x + (1ull << b)) < M) x += 1ull << b;
  const float aM = key_unorder((uint32_t)x);
  const double tp = (double)aM + 2.000001 * bkey[q];
  if (tid == 0 && isfinite(tp) && tp < (double)FLT_MAX) {
    float t = (float)tp;
    if ((double)t < tp) t = nextafterf(t, INFINITY);
    if (t < cut[q]) cut[q] = t;
  }
}

hipError_t launch_qbound(int mode, const float* Q, int64_t ld, const float* qn, int filter,
                         const unsigned* stats, const float* qr2i8, int nq, double* bkey,
                         hipStream_t st, const BoundArgs* bap) {
  if (nq <= 0) return hipSuccess;
  if (ld % 4 != 0) return hipErrorInvalidValue;
  const BoundArgs ba = bap ? *bap : make_bound_args(ld, filter);
#define VS_QB(MD) \
  hipLaunchKernelGGL(qbound_kernel<MD>, dim3(nq), dim3(64), 0, st, Q, ld, qn, ba, stats, qr2i8, nq, bkey)
  if (mode == MODE_IP)
    VS_QB(MODE_IP);
  else if (mode == MODE_L2)
    VS_QB(MODE_L2);
  else if (mode == MODE_COS)
    VS_QB(MODE_COS);
  else
    return hipErrorInvalidValue;
#undef VS_QB
  return hipGetLastError();
}

static hipError_t launch_qcut(const X1Args& a, Partials part, hipStream_t st) {
  const int nq = a.nqa;
  hipLaunchKernelGGL(qcut_kernel, dim3(nq), dim3(kQcutThreads), 0, st, part.key, part.id, part.P, part.KP,
                     x1_lane_len(), a.qcut_m, a.qbkey, nq, a.qcut);
  return hipGetLastError();
}


BoundArgs make_bound_args(int64_t ld, int filter) {
  BoundArgs ba;
  ba.filter = filter;
  const double u = std::ldexp(1.0, -23);
  const double n = (double)ld + 1.0;
  ba.gam = filter == FILTER_I8 ? 6.0 * std::ldexp(1.0, -24) : n * u / (1.0 - n * u);
  // the stored norms are fp32 sums of ld squares: they undercount by at most
  // ~gam(ld), whatever the plane
  ba.norm_inf = 2.0 * (n * u / (1.0 - n * u));
  return ba;
}

BoundArgs make_bound_args_l2aug(int64_t ld, const L2Aug& g, int filter) {
  const bool i8 = filter == FILTER_I8;
  BoundArgs ba = make_bound_args(ld + (i8 ? g.m : kAugBf16), filter);
  ba.l2aug = 1;
  const double c = i8 ? (double)g.C : (double)g.Cb;
  ba.aug_q2 = (i8 ? (double)g.m : (double)kAugBf16) * c * c;
  ba.aug_nref = (double)g.nref;
  return ba;
}

}  // namespace vs
