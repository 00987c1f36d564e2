// Internal declarations shared by vs_kernels.hip (device code + launchers) and
// vs_api.hip (the C-ABI).  Nothing here is part of the public ABI.
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdint>

namespace vs {

// Score modes of the fused kernels.  Every mode is reduced to a "key" where
// smaller is better, so one list discipline serves all of them:
//   IP : key = -<q,x>                        (faiss knn_inner_product, CMin heap)
//   L2 : key = (|q|^2 + |x|^2) - 2<q,x>, <0 -> 0 (faiss knn_L2sqr BLAS branch)
//   L2D: key = sum (x-q)^2                   (faiss knn_L2sqr sequential branch, nq < 20)
//   COS: key = -(<q,x> * rq * rx)             (pgvector 1 - (a <=> b))
enum Mode : int { MODE_IP = 0, MODE_L2 = 1, MODE_COS = 2, MODE_L2D = 3 };

// GEMM tile geometry (fp32 MFMA path): 128 database rows x 128 queries per
// workgroup, K staged 32 floats at a time through LDS.
constexpr int kBN = 128;
constexpr int kBQ = 128;
constexpr int kBK = 32;
// Row storage stride (floats) is a multiple of kBK; capacity keeps >= kBQ rows of
// zeroed slack past ntotal and is a multiple of kRowPad, so every tile load of
// the GEMM (database tiles and self-join query tiles) stays inside the buffer.
constexpr int kRowPad = 256;
// The GEMV (small batch) path handles up to this many queries per launch.
constexpr int kGemvMaxQ = 8;
// faiss's distance_compute_blas_threshold: a search CALL with fewer queries runs
// the sequential branch (L2 as the direct sum of squares).
constexpr int kBlasThreshold = 20;
// The skinny MFMA (small batch) path handles up to this many queries per launch.
constexpr int kSkinnyMaxQ = 32;

__host__ __device__ inline uint16_t f32_to_bf16_rne(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu))  // NaN stays a (quiet) NaN
    return (uint16_t)((u >> 16) | 0x0040u);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// Merge-buffer record: key + local row id (int32; a shard never holds 2^31 rows).
struct Partials {
  float* key = nullptr;
  int* id = nullptr;
  int P = 0;   // lists per query
  int KP = 0;  // entries per list
  int KL = 0;  // for launch_merge_partials: entries stored per list when fewer
               // than the merge keeps (0 = KP; a multiple of 4)
};

// ---- launchers (return the launch status; all asynchronous on `st`) -------
// Fused MFMA distance + top-k over database tiles, writing 2*nsplit lists/query.
// X / Q are fp32 (esize 4) or bf16 (esize 2) rows of stride ld elements.
// With `qlist`, query slot s of the (nq_pad-row) batch is row qlist[s] of Q (and
// of qaux; self row self0 + qlist[s]), only slots s < *qcount are computed
// (query tiles past the device-side count return at once), lists indexed by slot.
// With fkey/fid (inner product, KP = 64): only rows strictly after the query's
// floor (fkey, fid) in (key, row) order enter (floors indexed like qaux).
hipError_t launch_gemm_topk(int KP, int mode, const void* X, const float* xaux, const void* Q,
                            const float* qaux, int64_t ld, int esize, int ntotal, int nq_pad,
                            int nsplit, int64_t self0, Partials part, hipStream_t st,
                            const int* qlist = nullptr, const int* qcount = nullptr,
                            const float* fkey = nullptr, const int* fid = nullptr);
// Streaming (HBM-bound) distance + top-k for nq <= kGemvMaxQ.
// X fp32 or bf16 rows; Q always fp32 (values already rounded for bf16 indexes).
// With fkey/fid (inner product, KP = 64): the floor of each query, as in
// launch_gemm_topk; `run` (device, optional): every block exits when *run == 0.
hipError_t launch_gemv_topk(int KP, int mode, int nq, const void* X, int esize, const float* Q,
                            int64_t ld, int ntotal, int nblocks, Partials part, hipStream_t st,
                            const float* fkey = nullptr, const int* fid = nullptr,
                            const int* run = nullptr);
// Small-batch MFMA path (nq <= kSkinnyMaxQ, KP <= 32, IP or L2 via norms):
// one list per query per block, part.P == nblocks.
// The deep bf16 stage for a few gathered queries (device-side count; the
// kernel exits when it is 0 or above skinny_plane_max_queries()): lane lists
// of 8 in the x1 layout [slot][part.P][part.KP] from the tile-major bf16 plane
// (ld = the plane's K in elements) and the gathered query plane's tile 0.
// filter FILTER_I8: the int8 plane with the x1 pass's keys (qs: the queries'
// scales, xs: the rows' factors).
hipError_t launch_skinny_plane(int filter, const void* XH, const void* QH, int64_t ld, int ntotal,
                               const int* qcount, const float* qs, const float* xs, Partials part,
                               hipStream_t st, int nq_hint = 0);
int skinny_plane_max_queries();
// qcount (optional, device): the kernel does nothing when *qcount is 0 (the
// staged engine's last stage over a gathered batch, usually empty)
hipError_t launch_skinny_topk(int KP, int mode, int nq, const void* X, int esize,
                              const float* xaux, const void* Q, const float* qaux, int64_t ld,
                              int ntotal, int nblocks, Partials part, hipStream_t st,
                              const int* qcount = nullptr);
// The filter pass of the filter-and-verify engine (vs_gemm_x1.hip): one MFMA
// product per fp32 product over a low-precision "filter plane" of rows and
// queries: bf16 (RNE) on v_mfma_f32_32x32x16_bf16, or int8 with one fp32 scale
// per row (code = rint(x / s), s = max|x| / 127) on v_mfma_i32_32x32x32_i8
// (twice the bf16 rate, exact int32 sums, half the bytes per element).
enum Filter : int { FILTER_BF16 = 0, FILTER_I8 = 1 };
inline int filter_bytes(int filter) { return filter == FILTER_I8 ? 1 : 2; }
// Filter planes are stored TILE-MAJOR: [tile of 256 rows][64-B step][256
// rows][64 B], so the bytes one filter-pass step reads from a tile (256 rows x
// 64 B) are one contiguous 16-KB block and every DMA piece is 1 KB of
// consecutive bytes (whole 128-B lines; cdna_hip_programming.md: fragment-
// shaped pieces of half lines cost the TA twice).  `ldb` = bytes per row, a
// multiple of 64.  Any row range of a capacity that is a multiple of 256 rows
// lives inside the same prefix of tiles whatever the capacity.
__host__ __device__ inline int64_t plane_offset(int64_t row, int64_t byte, int64_t ldb) {
  return ((row >> 8) * (ldb >> 6) + (byte >> 6)) * 16384 + (row & 255) * 64 + (byte & 63);
}
// Per-launch timing hook of the filter pass (vs_api.hip): x1_launch brackets
// every pass launch with begin/end; `dominant` is false for the list launch of
// a pass that dumps (its spans are named apart from the dump launches').
struct X1Timing {
  // share: the launch's part of the pass's database tiles
  virtual void begin(hipStream_t st, bool dominant, double share) = 0;
  virtual void end(hipStream_t st) = 0;
  virtual ~X1Timing() = default;
};
struct X1Args {
  X1Timing* timing = nullptr;
  int qskip = 0;  // gathered stage: counts <= qskip are skinny_plane_topk's (x1 exits)
  int filter = FILTER_BF16;
  const void* XH = nullptr;      // database plane, tile-major (plane_offset)
  const float* xs = nullptr;     // int8: per-row factor s_x (IP) or s_x / |x| (COS)
  const float* xgmax = nullptr;  // int8: launch_group_max of xs (capacity rows)
  const float* xgmin = nullptr;  // int8: the group minima of xs over rows < ntotal
  // Dump launches (vs_gemm_x1.hip header): after the pass's first launch the
  // cuts are set and the later launches store the blocks below them
  bool dump = false;
  float* qcut = nullptr;         // per query (nqa): the cut, set after the first launch
  const double* qbkey = nullptr; // per query: the verification's bound B (x1_qcut)
  int qcut_m = 0;                // the M of the verification
  int* dcount = nullptr;         // [nq_pad][P] dumps per lane list (zeroed before the pass)
  int* dslot = nullptr;          // [nq_pad][P][dR][2] dumped (row, raw sum) pairs
  int dR = 0;                    // dump slots per lane list and segment
  unsigned long long* dstats = nullptr;  // [2] dumps replayed, lists out of slots
  const float* xaux = nullptr;   // per-row norms (L2) or 1/|x| (COS)
  const void* QH = nullptr;      // query plane, tile-major (self-join: the stored plane)
  int qtile0 = 0;                // QH's tile of query tile 0 (self-join: self0 / 256)
  const float* qs = nullptr;     // int8: per-query factor s_q (IP) or s_q / |q| (COS)
  const float* qaux = nullptr;   // per-query aux, nqa entries (padding queries read 0)
  int nqa = 0;
  int64_t ld = 0;                // elements per row, a multiple of 64
  int ntotal = 0;
  int nq_pad = 0;                // multiple of kX1Q
  int nsplit = 1;
  int64_t self0 = -1;
  const int* qrow = nullptr;     // per-query excluded row (-1 none), else self0 + q
  const int* qcount = nullptr;   // gathered batch: device-side query count
};
constexpr int kX1Q = 256;  // queries (and database rows) per x1 tile
// int8 sums stay exact in int32 up to this many elements per row.
constexpr int64_t kI8MaxLd = 131072;
// Candidates merged from the lane lists for `need` exact entries (24, 32, 64 or
// 128; 0 = not served by the filter engine).
int x1_list_len(int need);
// Entries per lane list of the filter pass (8).
int x1_lane_len();
// Diagnostic: the per-segment cycle sums of a VS_X1_STAMP build (26 values:
// [2 groups][9 segments + 3 epilogue counts] + steps per group); zeros in a
// real build.
hipError_t x1_stamps(unsigned long long* out, int reset);
// Writes 4*nsplit lists of part.KP entries per query (nq_pad queries), each holding
// x1_lane_len() entries and empty padding.  *ndispatch = kernel launches used.
hipError_t launch_gemm_topk_x1(int mode, const X1Args& a, Partials part, hipStream_t st,
                               int* ndispatch);
// Bound constants of the verification (vs_gemm_x1.hip).
struct BoundArgs {
  int filter = FILTER_BF16;
  double gam = 0.0;       // relative error of the filter's own arithmetic (bf16: fp32
                          // accumulation of ld + 1 terms, n u / (1 - n u), u = 2^-23;
                          // int8: exact int32 sum, three fp32 roundings of the scaling)
  double norm_inf = 0.0;  // relative undercount of the stored fp32 norms
  // L2 on the int8 plane (the augmented inner product, launch_quantize_i8_l2aug):
  // the bound is the inner-product bound of the augmented vectors, mapped to
  // the L2 key; aug_q2 = m C^2, what the augmentation adds to every |q|^2
  int l2aug = 0;
  double aug_q2 = 0.0;
  double aug_nref = 0.0;  // the augmentation's reference norm (launch_l2aug_map)
  // the pass multiplied the fp32 rows and queries themselves (the exact
  // engine's fp32 GEMM, the staged engine's last stage): no residuals, only the
  // fp32 accumulation (gam as for bf16 products) and the key's own roundings
  int rows_exact = 0;
};
BoundArgs make_bound_args(int64_t ld, int filter);
// The augmentation of an L2 index's int8 plane (launch_quantize_i8_l2aug).
struct L2Aug {
  int m = 0;          // int8 extra columns (a multiple of 64)
  float C = 0.0f;     // the queries' extra entry (int8 plane)
  float nref = 0.0f;  // reference norm: the rows' extra entries sum to (nref - n_x) / (2 C)
  float Cb = 0.0f;    // bf16 plane: the queries' extra entry (C's power of two, exact in bf16)
};
// Extra columns of an L2 index's augmented bf16 plane (bf16 has no per-row
// scale to keep the extra entries within: one 64-element block).
constexpr int kAugBf16 = 64;
// The bound constants for an L2 index's augmented int8 / bf16 plane.
BoundArgs make_bound_args_l2aug(int64_t ld, const L2Aug& g, int filter = FILTER_I8);
// out[0..3) = bits of max norms, max rn2, max rn2/norms over rows [0, n).
// accumulate: fold rows [0, n) into the maxima already in out (no reset).
hipError_t launch_bound_stats(const float* norms, const float* rn2, int64_t n, unsigned* out,
                              hipStream_t st, bool accumulate = false);
// rn2[r] = |x_r - bf16_rne(x_r)|^2 (rounded up) for fp32 rows [r0, r0+n).
hipError_t launch_resid_norms(const float* X, int64_t ld, int64_t r0, int64_t n, float* out,
                              hipStream_t st);
// int8 filter plane of fp32 rows [r0, r0+n) (stride ld): codes (int8,
// tile-major plane rows r0..), scale[r] = max|x_r| / 127 and, when rn2 != nullptr, rn2[r] = |x_r - scale
// * code_r|^2 rounded up (+inf for a row with a non-finite element).
// X: fp32 rows (xesize 4) or bf16 rows (xesize 2: a bf16 index's int8 plane).
hipError_t launch_quantize_i8(const void* X, int64_t ld, int64_t r0, int64_t n, int8_t* codes,
                              float* scale, float* rn2, hipStream_t st, int xesize = 4);
// L2 as an inner product ("int8 L2"): ranking rows by the faiss
// L2 key |q|^2 + |x|^2 - 2 q.x is ranking them by q.x + (nref - n_x) / 2 =
// x'.q' with x' = [x, e_1 .. e_m], sum_j C e_j = (nref - n_x) / 2 (n_x the
// stored norm, nref a constant of the index: the largest norm of its first
// rows, so the scores of the best rows stay positive and the extra entries
// small), and q' = [q, C .. C].  Rows (norms != nullptr): the codes of x'
// (plane rows of ld + m bytes, the extra columns at [ld, ld + m)), s =
// max(max|x|, |E| / m) / 127 with E = (nref - n_x) / (2 C), the extra codes an
// even split of T = rint(E / s) (the conceptual e_j are those codes' values
// plus an even share of the remainder, so the residual of the extra block is
// |E - s T|^2 / m), rn2 = |x' - plane(x')|^2 and anorm = |x'|^2, both rounded
// up.  Queries (norms == nullptr): extra codes c and s = C / c with c =
// min(127, floor(127 C / max|q|)) (so s * c = C up to one rounding), rn2 =
// |q' - plane(q')|^2 rounded up.
hipError_t launch_quantize_i8_l2aug(const float* X, int64_t ld, int64_t r0, int64_t n,
                                    const L2Aug& g, const float* norms, int8_t* codes,
                                    float* scale, float* rn2, float* anorm, hipStream_t st);
// The same augmentation on the bf16 plane (plane rows of ld + kAugBf16
// elements): rows (norms != nullptr) get kAugBf16 equal extra entries
// bf16(E / kAugBf16), E = (nref - n_x) / (2 Cb) (the conceptual entries add an
// even share of E minus their sum: residual |E - sum|^2 / kAugBf16), rn2 =
// |x' - plane(x')|^2 and anorm = |x'|^2 rounded up; queries (norms == nullptr)
// get Cb (exact: a power of two).
hipError_t launch_bf16_plane_l2aug(const float* X, int64_t ld, int64_t r0, int64_t n,
                                   const L2Aug& g, const float* norms, uint16_t* plane, float* rn2,
                                   float* anorm, hipStream_t st);
// The augmentation's parameters from fp32 rows [r0, r0+n): C = the mean of
// max|x| over the nonzero rows, nref = the largest norm, m = the extra columns
// that keep every row's extra entries within its own max|x|
// (|nref - n_x| / (2 C max|x|) at most), rounded up to 64, at least 64 (no
// nonzero row: C = 1).  Synchronises `st`.
hipError_t l2aug_params(const float* X, int64_t ld, int64_t r0, int64_t n, const float* norms,
                        L2Aug* out, hipStream_t st);
// Lane lists of an augmented pass -> L2 keys: key = max(0, fl(fl(|q|^2 + nref)
// + 2 key)) for every entry with a row (the map is monotone, so the lists stay
// sorted and every floor stays a floor), and the cuts likewise (-FLT_MAX kept).
hipError_t launch_l2aug_map(float* key, const int* id, int64_t per_query, int nq,
                            const float* qn, float nref, float* qcut, hipStream_t st);
// A later filter stage's gathered batch: dst[s] = src[gl[s]] (rows of stride
// ld), daux[s] = aux[gl[s]], drow[s] = self0 + gl[s] (or -1) for s < *count,
// zero rows / 0 / -1 for the other slots of [0, nslot).
hipError_t launch_gather_queries(const float* src, int64_t ld, const float* aux, const int* gl,
                                 const int* count, int nslot, int64_t self0, float* dst,
                                 float* daux, int* drow, hipStream_t st);
// acc[0] += n, acc[1] += *count.
hipError_t launch_add_counts(const int* count, int n, unsigned long long* acc, hipStream_t st);
// out[j] = outer[inner[j]] for j < *count (j < n).
hipError_t launch_compose_list(const int* outer, const int* inner, const int* count, int n,
                               int* out, hipStream_t st);
// *out = clamp(*count - w0, 0, cap): the device-side count of one slot window
// [w0, w0 + cap) of a gathered batch.
hipError_t launch_window_count(const int* count, int w0, int cap, int* out, hipStream_t st);
// out[2 g + b] = max of f over the rows of 32-row group g whose bit 2 is b
// (the int8 filter's per-lane factor bound), n a multiple of 32.
hipError_t launch_group_max(const float* f, int64_t n, float* out, hipStream_t st,
                            int64_t nvalid = 0, float* outmin = nullptr);
// out[i] = a[i] * b[i] (the int8 cosine's folded factors s / |x|).
hipError_t launch_mul_arrays(const float* a, const float* b, int64_t n, float* out,
                             hipStream_t st);
// Checks and rescores the filter candidates: Dk/Ik hold the KF best approximate
// keys of each query (ascending, local rows), `lists` the filter pass's lane
// lists (L entries each) for their floors; writes sorted exact lists of KP
// entries (okey/oid) and fail[q] = 1 where the exact engine must redo query q.
// qsc: the queries' int8 scales (int8 filter; null for bf16).
hipError_t launch_verify_rescore(int mode, int nq, int KF, int M, const float* Dk,
                                 const int64_t* Ik, const void* X, const float* xn,
                                 const float* Q, const float* qn, int64_t ld, const BoundArgs& ba,
                                 const unsigned* stats, Partials lists, int L, float* okey,
                                 int* oid, int KP, int* fail, hipStream_t st,
                                 const float* qinv, const float* xinv, const float* qsc,
                                 const int* qcount = nullptr, const float* qcut = nullptr,
                                 int xesize = 4);
// Flagged queries (flags[i] != 0) -> ascending qlist[0 .. *count), all on the
// device; *total += count and *total_n += n when not null.
hipError_t launch_compact_flags(const int* flags, int n, int* list, int* count,
                                unsigned long long* total, unsigned long long* total_n,
                                hipStream_t st);
// Second verification of the queries qlist[0 .. *count) (device count, fixed
// grid): every lane-list entry below the smallest full-list floor (or below
// Dk's M-th key + 2 B when that is smaller; Dk = the merged approximate keys,
// [nq][KF], Ik its rows) is rescored
// exactly (up to kWideCap per query) and the condition re-checked on that wider
// set; passing queries get their sorted exact list in okey/oid and fail[q] = 0.
// okey/oid hold on entry the first check's exact keys of Ik (KP <= 64), which
// are reused instead of read again.  sizes (optional): += the wide-set entries
// and the rescored ones.
constexpr int kWideCap = 4096;
// The most candidates (KF) the verification rescores per query, and the longest
// exact list (KP) it writes: 1024 holds inner product's 2k - 1 for k <= 512
// (and k <= 1023 for L2 / cosine); past it the paged exact engine answers.
constexpr int kVerifyMaxKF = 1024;
// The KF (<= kVerifyMaxKF) lexicographically best (key, row) entries of every
// query's P lane lists of L entries (stride part.KP), ascending, into Dk/Ik
// [nq][KF] (the approximate merge when KF > 64; launch_merge_partials below).
hipError_t launch_select_lists(Partials part, int L, int nq, int KF, float* Dk, int64_t* Ik,
                               hipStream_t st, const int* qcount = nullptr);
// The same for KF <= 64 from lane lists of L = 8 (stride 8) by a bound from the
// lists' heads (P >= KF, P <= 512; select_heads_applies), else the list merge.
bool select_heads_applies(const Partials& part, int L, int KF);
hipError_t launch_select_heads(Partials part, int nq, int KF, float* Dk, int64_t* Ik,
                               hipStream_t st, const int* qcount = nullptr);

// Scratch chunks (vs_api.hip): device memory of at least `bytes` whose previous
// use the taker's stream `st` waits for; put records the chunk's last use on
// `st` and keeps it for the next taker.  scratch_trim frees the idle chunks of
// the current device (synchronising it).
struct ScratchChunk {
  void* p = nullptr;
  size_t size = 0;
  int dev = 0;
  hipEvent_t ev = nullptr;
  hipStream_t st = nullptr;  // the stream of its last use
};
hipError_t scratch_chunk_get(size_t bytes, hipStream_t st, ScratchChunk* out);
void scratch_chunk_put(const ScratchChunk& c, hipStream_t st);
void scratch_trim();
hipError_t launch_verify_wide(int mode, int nq_max, const int* qlist, const int* count, int KF,
                              int M, const void* X, const float* xn, const float* Q,
                              const float* qn, int64_t ld, const BoundArgs& ba,
                              const unsigned* stats, Partials lists, int L, float* okey, int* oid,
                              int KP, int* fail, hipStream_t st, const float* qinv,
                              const float* xinv, const float* qsc, const float* Dk,
                              const int64_t* Ik, unsigned long long* sizes = nullptr,
                              const float* qcut = nullptr, int xesize = 4);
// Query cuts and dump launches of the filter pass (vs_gemm_x1.hip, "Query
// cuts"): bkey[q] = the verification's bound B of query q; x1_dump_applies:
// the pass of this mode and plane has a dump form (launch_gemm_topk_x1 then
// sets the cuts after its first launch and dumps in the others; the host runs
// launch_x1_replay after it, and the verification must get the same cuts).
hipError_t launch_qbound(int mode, const float* Q, int64_t ld, const float* qn, int filter,
                         const unsigned* stats, const float* qr2i8, int nq, double* bkey,
                         hipStream_t st, const BoundArgs* ba = nullptr);
bool x1_dump_applies(int mode, int filter);
int x1_dump_slots();  // the most dump slots per lane list worth allocating
bool x1_pass_dumps(int ntotal, int nsplit);  // a pass this long has dump launches
// a.dstats[0] += dumps replayed, a.dstats[1] += lane lists out of slots
// (launch_gemm_topk_x1 calls it between its segments of dump launches)
hipError_t launch_x1_replay(const X1Args& a, Partials part, hipStream_t st);
// Lists -> final (D, I) rows of k entries each (row stride ldo), labels offset by id_base.
// Inner product applies faiss's tie rule unless `raw` (plain lexicographic
// (key, label) order, the per-shard half of an exact sharded merge).  With
// `qlist`, list q belongs to query qlist[q] (emitted to that row) and only
// q < *qcount are merged (device-side count; the grid covers nq).
hipError_t launch_merge_partials(int mode, Partials part, int nq, int k, int64_t id_base,
                                 float min_score, float* D, int64_t* I, int64_t ldo,
                                 hipStream_t st, int raw = 0, const int* qlist = nullptr,
                                 const int* qcount = nullptr);
// Shard lists [nparts][nq][k_in] (scores, int64 labels) -> [nq][k].
hipError_t launch_merge_parts(int mode, const float* Dp, const int64_t* Ip, int nparts,
                              int nq, int k_in, int k, float* D, int64_t* I, hipStream_t st);
// The exact-key stream (vs_exact.hip): for the gathered slots
// slots[s0 .. s0 + min(*count - s0, nslot)) of a query batch whose rows sit at
// Q + slot * ld (aux values qaux[slot]: |q|^2 for L2, 1/|q| for cosine; qrow[slot]:
// the row to exclude, or -1; qrow may be null), the top-KP of every row by the
// rescoring's exact key (fp64 sums, vs_gemm_x1.hip exact_key), as part.P lists
// per slot (part.P row blocks).  NQ queries per group: exact_stream_nq(ld)
// (0: ld too large for the LDS staging).
struct ExactStreamArgs {
  const float* X = nullptr;     // fp32 rows [ntotal][ld]
  const float* xn = nullptr;    // |x|^2 (L2)
  const float* xinv = nullptr;  // 1/|x| (cosine)
  int64_t ld = 0;
  int ntotal = 0;
  const float* Q = nullptr;
  const float* qaux = nullptr;
  const int* qrow = nullptr;
  const int* slots = nullptr;
  const int* count = nullptr;
  int s0 = 0, nslot = 0;
  // per query (indexed like slots' entries): only entries lexicographically
  // after (fkey, fid) enter (a page of the paged engine); null: no floor
  const float* fkey = nullptr;
  const int* fid = nullptr;
};
int exact_stream_nq(int64_t ld);
hipError_t launch_exact_stream(int KP, int mode, const ExactStreamArgs& a, Partials part,
                               hipStream_t st);
// The paged exact engine (vs_support.hip, "paged exact engine"; vs_api.hip
// run_paged).  Dacc/Iacc [n][KA]: the pages side by side (scores, local rows).
// page_init: member/active flags (every q < n, or gl[0 .. *gc) of zeroed rows)
// and the first page's floor (-inf, -1) for fkey/fid[0 .. nfloor).
hipError_t launch_page_init(int n, int nfloor, const int* gl, const int* gc, int* member,
                            int* active, float* fkey, int* fid, hipStream_t st);
// After page `page`: active[q] = query q needs the next page (its page was full
// and it has fewer than k entries, or `rule` and the k-th key's run of ties
// reaches the page's end below 2k - 1), fkey/fid = its floor (+inf when not).
hipError_t launch_page_step(const float* Dacc, const int64_t* Iacc, int64_t KA, int page, int n,
                            int64_t k, int rule, int mode, int* active, float* fkey, int* fid,
                            hipStream_t st);
// *out = *count > 0 ? n : 0 (the device-side count of a GEMV page's lists).
hipError_t launch_page_gate(const int* count, int n, int* out, hipStream_t st);
// The member queries' k outputs (faiss's inner-product rule when `rule`), rows
// q * k of D / I, labels + id_base, min_score applied as merge_partials does.
hipError_t launch_page_finish(int mode, float* Dacc, int64_t* Iacc, int64_t KA, int n, int64_t k,
                              int rule, const int* member, int64_t id_base, float min_score,
                              float* D, int64_t* I, hipStream_t st);
// out[r] = sum_j X[r][j]^2 for rows [r0, r0+n) (fp32 or bf16 rows).
hipError_t launch_row_norms(const void* X, int esize, int64_t ld, int64_t r0, int64_t n,
                            float* out, hipStream_t st);
// Pitched conversions: fp32 -> bf16 (round to nearest even, NaN kept) with zero
// padding of columns [cols, ldo); bf16 -> fp32 (exact widening); fp32 -> fp32
// rounded through bf16 (the value a bf16 index stores).
hipError_t launch_f32_to_bf16(const float* in, int64_t ldi, uint16_t* out, int64_t ldo,
                              int64_t rows, int64_t cols, hipStream_t st);
// bf16 plane (tile-major) of fp32 rows [r0, r0+n) of stride ld (ld elements
// per plane row, RNE).
hipError_t launch_bf16_plane(const float* X, int64_t ld, int64_t r0, int64_t n, uint16_t* plane,
                             hipStream_t st);
// Zeroes plane rows [r0, r0+n) of a tile-major plane with ldb bytes per row.
hipError_t launch_plane_zero_rows(char* plane, int64_t ldb, int64_t r0, int64_t n, hipStream_t st);
hipError_t launch_bf16_to_f32(const uint16_t* in, int64_t ldi, float* out, int64_t ldo,
                              int64_t rows, int64_t cols, hipStream_t st);
hipError_t launch_round_bf16(float* x, int64_t n, hipStream_t st);
// out[r] = 1/sqrt(norm[r]) (double-precision rsqrt rounded to float).
hipError_t launch_rsqrt(const float* norm, int64_t n, float* out, hipStream_t st);
// Counter-based synthetic rows into a pitched fp32 or bf16 buffer (zero padding d..ldo).
hipError_t launch_fill_synthetic(void* out, int esize, int64_t rows, int64_t d, int64_t ldo,
                                 uint64_t seed, int64_t row0, hipStream_t st);
// Same generator for an explicit list of generator row numbers (device int64).
hipError_t launch_fill_synthetic_ids(void* out, int esize, const int64_t* ids, int64_t rows,
                                     int64_t d, int64_t ldo, uint64_t seed, hipStream_t st);
// Fill n (D, I) pairs with the empty-result sentinel of `mode`.
hipError_t launch_fill_empty(int mode, float* D, int64_t* I, int64_t n, hipStream_t st);
// Stable compaction helper: copy the kept rows of [src0, src0+n) into tmp,
// given the sorted removed-row list (device).  Also moves the norms.
// Rows are `rowbytes` long (multiple of 16).
// out[0 .. n) = 0 .. n-1 and *count = n (device): a gathered batch of every query.
hipError_t launch_iota(int* out, int n, int* count, hipStream_t st);
// Tombstones: rows[0 .. n) (device) filled with NaN elements and a NaN norm;
// the labels I[0 .. n) of a search (kernel rows + id_base) mapped to positions
// among the live rows (dead: the sorted tombstoned rows, ndead of them).
// scale (optional): the int8 plane's row factors, set to NaN too (the plane's
// keys of a tombstoned row are NaN and never enter a list).
hipError_t launch_fill_nan_rows(void* X, int64_t rowbytes, float* norms, int esize,
                                const int64_t* rows, int64_t n, hipStream_t st,
                                float* scale = nullptr);
hipError_t launch_label_map(int64_t* I, int64_t n, const int64_t* dead, int64_t ndead,
                            int64_t id_base, hipStream_t st);
hipError_t launch_gather_kept(const void* X, const float* norms, int64_t rowbytes, int64_t src0,
                              int64_t n, const int64_t* removed, int64_t nrem, void* tmp,
                              float* tmp_norms, hipStream_t st);

}  // namespace vs
