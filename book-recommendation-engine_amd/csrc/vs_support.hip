// vs_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the exact flat index.
//
// Semantics follow faiss-cpu 1.11.0 IndexFlat::search (not vendored; pinned at
// /root/reference/poetry.lock:866-867): exact top-k, squared L2 or inner
// product, ties broken by the lower label, k > ntotal padded with (neutral, -1).
// Every score is mapped to a key where smaller is better (vs_internal.h), and
// lists are ordered by (key, row) lexicographically — the order faiss's heaps
// produce with CMax/CMin::cmp2.
//
// Kernels
//   gemm_topk_f32   fp32 MFMA (v_mfma_f32_32x32x2_f32) Q.X^T tile with the top-k
//                   selection fused into the epilogue; large query batches,
//                   bounded by the fp32 matrix-core peak.
//   gemv_topk_f32   one streaming pass of the corpus for nq <= 8, bounded by HBM.
//   merge_*         per-query merge of partial lists (also the shard merge that
//                   follows the RCCL all-gather).
//   row_norms, rsqrt, fill_synthetic, fill_empty, gather_kept: support.
#include "vs_device.h"

namespace vs {

// ---------------------------------------------------------------------------
// Merge: one wave per query.  Each lane filters a strided slice of the
// candidates into its own register list, then the 64 lists are combined by a
// 6-round pairwise merge through LDS.  Output keys are mapped back to scores.
template <int KP, typename IdT>
__device__ __forceinline__ void wave_tree_merge(float (&lk)[KP], IdT (&li)[KP], float* sk,
                                                IdT* si, int lane, int nvalid = 64,
                                                int len0 = KP) {
  // sk/si: LDS [64][KP + 1] (the odd row stride spreads the active lanes' rows
  // over all banks; a stride of KP put every even lane on one bank); on return
  // lane 0 holds the merge of the 64 lists.  Only lanes < nvalid hold entries
  // (rounds past them are skipped), each at most len0 (the rest empty): a
  // round's lists hold at most `len` entries, so it writes and merges 2 len.
  constexpr int KS = KP + 1;
  // (KP = 64 keeps full-length rounds: the bounded form spills there)
  int len = KP <= 32 && len0 < KP ? len0 : KP;
  for (int step = 1; step < 64 && step < nvalid; step <<= 1) {
    const int lim = 2 * len < KP ? 2 * len : KP;
    if ((lane & (step - 1)) == 0) {
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        if (j >= lim) break;
        sk[lane * KS + j] = lk[j];
        si[lane * KS + j] = li[j];
      }
    }
    __syncthreads();
    if ((lane & (2 * step - 1)) == 0)
      merge2_sorted_n<KP, IdT>(sk + lane * KS, si + lane * KS, sk + (lane + step) * KS,
                               si + (lane + step) * KS, lk, li, lim);
    __syncthreads();
    len = lim;
  }
}

// faiss's inner-product tie rule on a lexicographic (key, label) list held in
// LDS (lane 0 only).  faiss's CMin heap keeps, at equal scores, the SMALLER label
// on top, so later better rows evict the smallest admitted labels; and
// heap_reorder emits equal scores in DESCENDING label order.  With v the k-th key,
// c the count strictly better, a_i the labels with key v (ascending) and g_i the
// number of better labels below a_i, faiss keeps a_{A-r} .. a_{A-1} where
// A = #{i : i + g_i < k} and r = k - c.  (L2's CMax heap needs no adjustment: it
// is exactly the lexicographic order.)  The candidate pool is the merged list;
// if its v-run was truncated at KP entries the result stays a valid tie order.
template <typename IdT>
__device__ void faiss_ip_tie_order(float* sk, IdT* si, int KP, int k) {
  int nv = 0;
  while (nv < KP && si[nv] >= 0) ++nv;
  const int m = nv < k ? nv : k;
  if (nv > k) {
    const float v = sk[k - 1];
    int c = 0;
    while (sk[c] < v) ++c;
    int t = 0;
    while (c + t < nv && sk[c + t] == v) ++t;
    int A = 0;
    for (int i = 0; i < t; ++i) {
      int g = 0;
      for (int j = 0; j < c; ++j) g += si[j] < si[c + i] ? 1 : 0;
      if (i + g < k) A = i + 1;
      else break;
    }
    const int r = k - c;
    for (int i = 0; i < r; ++i) {  // source index >= destination: forward copy is safe
      sk[c + i] = sk[c + A - r + i];
      si[c + i] = si[c + A - r + i];
    }
  }
  for (int s0 = 0; s0 < m;) {  // descending label inside equal keys
    int e = s0;
    while (e + 1 < m && sk[e + 1] == sk[s0]) ++e;
    for (int a = s0, b = e; a < b; ++a, --b) {
      const IdT tmp = si[a];
      si[a] = si[b];
      si[b] = tmp;
    }
    s0 = e + 1;
  }
}

__device__ __forceinline__ void emit_result(int mode, float key, int64_t id, int64_t id_base,
                                            float min_score, float* D, int64_t* I) {
  if (id < 0) {
    *D = (mode == MODE_L2 || mode == MODE_L2D) ? FLT_MAX : -FLT_MAX;
    *I = -1;
    return;
  }
  const float score = (mode == MODE_L2 || mode == MODE_L2D) ? key : -key;
  if (mode == MODE_COS && !(score >= min_score)) {
    *D = -FLT_MAX;
    *I = -1;
    return;
  }
  *D = score;
  *I = id + id_base;
}

// Multi-level list merge.  Every partial list is sorted (entry 0 best), so a wave
// loads one whole list per lane (vector loads, all in flight together) and
// tree-merges 64 lists in 6 rounds; levels repeat until one list per query is
// left, which is emitted as (D, I) rows (grid x = query, y = list group).
template <int KP>
__global__ __launch_bounds__(64) void merge_lists_kernel(
    const float* __restrict__ pkey, const int* __restrict__ pid, int P, int KL,
    float* __restrict__ okey,
    int* __restrict__ oid, int P2, int emit, int k, int mode, int raw, int64_t id_base,
    float min_score, float* __restrict__ D, int64_t* __restrict__ I, int64_t ldo,
    const int* __restrict__ qlist, const int* __restrict__ qcount) {
  __shared__ float sk[64 * (KP + 1)];
  __shared__ int si[64 * (KP + 1)];
  const int lane = threadIdx.x;
  const int q = blockIdx.x;
  const int g = blockIdx.y;
  if (qcount && q >= *qcount) return;  // gathered batch: slots past the count
  const int p = g * 64 + lane;
  float lk[KP];
  int li[KP];
  list_init<KP, int>(lk, li);
  if (p < P) {  // KL <= KP stored entries per list (a multiple of 4)
    const f32x4* ks = (const f32x4*)(pkey + ((int64_t)q * P + p) * KL);
    const int4* is = (const int4*)(pid + ((int64_t)q * P + p) * KL);
#pragma unroll
    for (int j = 0; j < KP / 4; ++j) {
      if (4 * j >= KL) break;
      const f32x4 kv = ks[j];
      const int4 iv = is[j];
      lk[4 * j + 0] = kv.x;
      lk[4 * j + 1] = kv.y;
      lk[4 * j + 2] = kv.z;
      lk[4 * j + 3] = kv.w;
      li[4 * j + 0] = iv.x;
      li[4 * j + 1] = iv.y;
      li[4 * j + 2] = iv.z;
      li[4 * j + 3] = iv.w;
    }
  }
  wave_tree_merge<KP, int>(lk, li, sk, si, lane, P - g * 64 < 64 ? P - g * 64 : 64, KL);
  if (!emit) {
    if (lane == 0) {
      float* ok = okey + ((int64_t)q * P2 + g) * KP;
      int* oi = oid + ((int64_t)q * P2 + g) * KP;
#pragma unroll
      for (int j = 0; j < KP; ++j) {
        ok[j] = lk[j];
        oi[j] = li[j];
      }
    }
    return;
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      sk[j] = lk[j];
      si[j] = li[j];
    }
    if (mode == MODE_IP && !raw) faiss_ip_tie_order<int>(sk, si, KP, k);
  }
  __syncthreads();
  const int64_t qe = qlist ? qlist[q] : q;  // output row
  if (lane < k) emit_result(mode, sk[lane], si[lane], id_base, min_score, D + qe * ldo + lane,
                            I + qe * ldo + lane);
}

template <int KP>
static hipError_t merge_levels(int mode, Partials part, int nq, int k, int64_t id_base,
                               float min_score, float* D, int64_t* I, int64_t ldo, int raw,
                               hipStream_t st, const int* qlist, const int* qcount) {
  const float* ck = part.key;
  const int* ci = part.id;
  int P = part.P;
  int KL = part.KL > 0 ? part.KL : KP;
  // one stream-ordered buffer for every level (each level writes its own
  // slice): one allocation and one free per merge
  size_t total = 0;
  for (int p = P; p > 64; p = (p + 63) / 64) total += (size_t)nq * ((p + 63) / 64) * KP;
  ScratchChunk chunk;
  hipError_t e = hipSuccess;
  if (total) e = scratch_chunk_get(total * (sizeof(float) + sizeof(int)), st, &chunk);
  float* okb = (float*)chunk.p;
  int* oib = (int*)(okb + total);
  while (P > 64 && e == hipSuccess) {
    const int P2 = (P + 63) / 64;
    float* ok = okb;
    int* oi = oib;
    okb += (size_t)nq * P2 * KP;
    oib += (size_t)nq * P2 * KP;
    hipLaunchKernelGGL((merge_lists_kernel<KP>), dim3(nq, P2), dim3(64), 0, st, ck, ci, P, KL, ok,
                       oi, P2, 0, k, mode, raw, id_base, min_score, D, I, ldo, qlist, qcount);
    e = hipGetLastError();
    ck = ok;
    ci = oi;
    P = P2;
    KL = KP;
  }
  if (e == hipSuccess) {
    hipLaunchKernelGGL((merge_lists_kernel<KP>), dim3(nq, 1), dim3(64), 0, st, ck, ci, P, KL,
                       (float*)nullptr, (int*)nullptr, 1, 1, k, mode, raw, id_base, min_score, D,
                       I, ldo, qlist, qcount);
    e = hipGetLastError();
  }
  scratch_chunk_put(chunk, st);
  return e;
}

// One sorted list of up to 128 entries per query (the verification's exact
// lists when inner product's rule reads 2k - 1 > 64 of them) -> (D, I) rows:
// faiss's rule on lane 0 over LDS, then the k outputs (k <= 128).
__global__ __launch_bounds__(64) void emit_list_kernel(
    const float* __restrict__ pkey, const int* __restrict__ pid, int KP, int k, int mode, int raw,
    int64_t id_base, float min_score, float* __restrict__ D, int64_t* __restrict__ I,
    int64_t ldo, const int* __restrict__ qlist, const int* __restrict__ qcount) {
  __shared__ float sk[kVerifyMaxKF];
  __shared__ int si[kVerifyMaxKF];
  const int lane = threadIdx.x;
  const int q = blockIdx.x;
  if (qcount && q >= *qcount) return;  // gathered batch: slots past the count
  for (int j = lane; j < kVerifyMaxKF; j += 64) {
    sk[j] = j < KP ? pkey[(int64_t)q * KP + j] : FLT_MAX;
    si[j] = j < KP ? pid[(int64_t)q * KP + j] : -1;
  }
  __syncthreads();
  if (lane == 0 && mode == MODE_IP && !raw) faiss_ip_tie_order<int>(sk, si, KP, k);
  __syncthreads();
  const int64_t qe = qlist ? qlist[q] : q;  // output row
  for (int j = lane; j < k; j += 64)
    emit_result(mode, sk[j], si[j], id_base, min_score, D + qe * ldo + j, I + qe * ldo + j);
}

hipError_t launch_merge_partials(int mode, Partials part, int nq, int k, int64_t id_base,
                                 float min_score, float* D, int64_t* I, int64_t ldo,
                                 hipStream_t st, int raw, const int* qlist, const int* qcount) {
  if (k < 1 || k > part.KP || nq < 0 || part.P < 1 || part.KL < 0 || part.KL > part.KP ||
      part.KL % 4 != 0)
    return hipErrorInvalidValue;
  if (nq == 0) return hipSuccess;
  if (part.KP > 64) {  // one sorted list per query only (the verification's output)
    if (part.KP > kVerifyMaxKF || part.P != 1 || (part.KL != 0 && part.KL != part.KP))
      return hipErrorInvalidValue;
    hipLaunchKernelGGL(emit_list_kernel, dim3(nq), dim3(64), 0, st, part.key, part.id, part.KP, k,
                       mode, raw, id_base, min_score, D, I, ldo, qlist, qcount);
    return hipGetLastError();
  }
  switch (part.KP) {
    case 8:
      return merge_levels<8>(mode, part, nq, k, id_base, min_score, D, I, ldo, raw, st, qlist, qcount);
    case 16:
      return merge_levels<16>(mode, part, nq, k, id_base, min_score, D, I, ldo, raw, st, qlist, qcount);
    case 32:
      return merge_levels<32>(mode, part, nq, k, id_base, min_score, D, I, ldo, raw, st, qlist, qcount);
    case 64:
      return merge_levels<64>(mode, part, nq, k, id_base, min_score, D, I, ldo, raw, st, qlist, qcount);
    default:
      return hipErrorInvalidValue;
  }
}

template <int KP>
__global__ __launch_bounds__(64) void merge_parts_kernel(const float* __restrict__ Dp,
                                                         const int64_t* __restrict__ Ip,
                                                         int nparts, int nq, int k_in, int k,
                                                         int mode, float* __restrict__ D,
                                                         int64_t* __restrict__ I) {
  __shared__ float sk[64 * (KP + 1)];
  __shared__ int64_t si[64 * (KP + 1)];
  const int lane = threadIdx.x;
  const int q = blockIdx.x;
  const bool asc = (mode == MODE_L2 || mode == MODE_L2D);
  float lk[KP];
  int64_t li[KP];
  list_init<KP, int64_t>(lk, li);
  const int64_t n = (int64_t)nparts * k_in;
  for (int64_t c = lane; c < n; c += 64) {
    const int p = (int)(c / k_in), j = (int)(c % k_in);
    const int64_t off = ((int64_t)p * nq + q) * k_in + j;
    const int64_t id = Ip[off];
    if (id >= 0) {
      const float s = Dp[off];
      list_insert<KP, int64_t>(lk, li, asc ? s : -s, id);
    }
  }
  wave_tree_merge<KP, int64_t>(lk, li, sk, si, lane);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < KP; ++j) {
      sk[j] = lk[j];
      si[j] = li[j];
    }
    if (!asc) faiss_ip_tie_order<int64_t>(sk, si, KP, k);
  }
  __syncthreads();
  if (lane < k) emit_result(asc ? MODE_L2 : MODE_IP, sk[lane], si[lane], 0, 0.0f,
                            D + (int64_t)q * k + lane, I + (int64_t)q * k + lane);
}

__global__ void merge_parts_big_kernel(const float* __restrict__ Dp,
                                       const int64_t* __restrict__ Ip, int nparts, int nq,
                                       int64_t k_in, int64_t need, int64_t k, int asc,
                                       float* __restrict__ sk, int64_t* __restrict__ si,
                                       float* __restrict__ D, int64_t* __restrict__ I);

hipError_t launch_merge_parts(int mode, const float* Dp, const int64_t* Ip, int nparts, int nq,
                              int k_in, int k, float* D, int64_t* I, hipStream_t st) {
  if (k < 1 || nq < 0 || nparts < 1 || k_in < 1) return hipErrorInvalidValue;
  if (nq == 0) return hipSuccess;
  // the pool keeps the lexicographically best `need` entries of all parts: k for
  // L2; for inner product the 2k-1 that faiss's tie rule reads
  const bool asc = (mode == MODE_L2 || mode == MODE_L2D);
  if ((!asc && 2 * k - 1 > 64) || k > 64) {  // beyond one 64-entry list
    if (nparts > 64) return hipErrorInvalidValue;
    const int64_t need = asc ? (int64_t)k : 2 * (int64_t)k - 1;
    ScratchChunk chunk;
    hipError_t e = scratch_chunk_get((size_t)nq * need * (sizeof(float) + sizeof(int64_t)), st,
                                     &chunk);
    if (e != hipSuccess) return e;
    int64_t* si = (int64_t*)chunk.p;
    float* sk = (float*)(si + (size_t)nq * need);
    hipLaunchKernelGGL(merge_parts_big_kernel, dim3((nq + 63) / 64), dim3(64), 0, st, Dp, Ip,
                       nparts, nq, (int64_t)k_in, need, (int64_t)k, asc ? 1 : 0, sk, si, D, I);
    e = hipGetLastError();
    scratch_chunk_put(chunk, st);
    return e;
  }
  const int need = asc ? k : 2 * k - 1;
  const int KP = need <= 8 ? 8 : need <= 16 ? 16 : need <= 32 ? 32 : 64;
  switch (KP) {
#define VS_MERGEP_CASE(KPV)                                                                   \
  case KPV:                                                                                  \
    hipLaunchKernelGGL((merge_parts_kernel<KPV>), dim3(nq), dim3(64), 0, st, Dp, Ip, nparts, \
                       nq, k_in, k, mode, D, I);                                             \
    break;
    VS_MERGEP_CASE(8)
    VS_MERGEP_CASE(16)
    VS_MERGEP_CASE(32)
    VS_MERGEP_CASE(64)
#undef VS_MERGEP_CASE
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The paged exact engine (vs_api.hip run_paged): any k, every metric.  A
// query's answer is read off its lexicographic (key, row) order in pages of 64
// entries, page p + 1 computed by the FLOOR form of the exact kernels (entries
// strictly after page p's last one).  The pages of a window of n queries land
// side by side in Dacc/Iacc [n][KA] (scores and local rows; -1 past the end).
//
// page_init: member[q] = the query belongs to this call (every q < n, or the
// gathered ones gl[0 .. *gc), whose member/active rows the host zeroed before),
// active[q] = member[q], floor (-inf, -1) (page 1 admits every row).
__global__ __launch_bounds__(256) void page_init_kernel(int n, int nfloor,
                                                        const int* __restrict__ gl,
                                                        const int* __restrict__ gc,
                                                        int* __restrict__ member,
                                                        int* __restrict__ active,
                                                        float* __restrict__ fkey,
                                                        int* __restrict__ fid) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < nfloor) {
    fkey[j] = -INFINITY;
    fid[j] = -1;
  }
  if (gl) {
    if (j < *gc) {
      member[gl[j]] = 1;
      active[gl[j]] = 1;
    }
  } else if (j < n) {
    member[j] = 1;
    active[j] = 1;
  }
}

hipError_t launch_page_init(int n, int nfloor, const int* gl, const int* gc, int* member,
                            int* active, float* fkey, int* fid, hipStream_t st) {
  const int m = n > nfloor ? n : nfloor;
  if (m <= 0) return hipSuccess;
  if ((gl == nullptr) != (gc == nullptr)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(page_init_kernel, dim3((m + 255) / 256), dim3(256), 0, st, n, nfloor, gl, gc,
                     member, active, fkey, fid);
  return hipGetLastError();
}

// After page `page` of the active queries: does query q need the next page?
// Only when the page came back full (64 entries: the order has more rows) and
// the answer needs more entries: fewer than k so far, or — faiss's
// inner-product rule (`rule`), which reads the k-th key's run of equal keys up
// to 2k - 1 entries (faiss_ip_tie_order) — the run reaches the page's end.
// Then the floor is the page's last entry; otherwise (+inf, INT_MAX), which
// empties a query's list in a GEMV page (its lists are computed for every query).
__global__ __launch_bounds__(256) void page_step_kernel(const float* __restrict__ Dacc,
                                                        const int64_t* __restrict__ Iacc,
                                                        int64_t KA, int page, int n, int64_t k,
                                                        int rule, int l2, int* __restrict__ active,
                                                        float* __restrict__ fkey,
                                                        int* __restrict__ fid) {
  const int q = blockIdx.x * 256 + threadIdx.x;
  if (q >= n) return;
  bool more = false;
  if (active[q]) {
    const float* d = Dacc + (int64_t)q * KA;
    const int64_t* i = Iacc + (int64_t)q * KA;
    const int64_t cnt = (int64_t)(page + 1) * 64;  // entries so far when the page is full
    const bool full = i[cnt - 1] >= 0;
    more = full && cnt < KA &&
           (cnt < k || (rule && cnt < 2 * k - 1 && d[cnt - 1] == d[k - 1]));
    if (more) {
      fkey[q] = l2 ? d[cnt - 1] : -d[cnt - 1];  // score -> key
      fid[q] = (int)i[cnt - 1];
    }
  }
  if (!more) {
    fkey[q] = INFINITY;
    fid[q] = INT_MAX;
  }
  active[q] = more ? 1 : 0;
}

hipError_t launch_page_step(const float* Dacc, const int64_t* Iacc, int64_t KA, int page, int n,
                            int64_t k, int rule, int mode, int* active, float* fkey, int* fid,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (KA % 64 != 0 || (int64_t)(page + 1) * 64 > KA || k < 1) return hipErrorInvalidValue;
  const int l2 = (mode == MODE_L2 || mode == MODE_L2D) ? 1 : 0;
  hipLaunchKernelGGL(page_step_kernel, dim3((n + 255) / 256), dim3(256), 0, st, Dacc, Iacc, KA,
                     page, n, k, rule, l2, active, fkey, fid);
  return hipGetLastError();
}

// *out = n when *count > 0, else 0 (a GEMV page's lists exist for every query
// of its window, or for none when its launch exited).
__global__ void page_gate_kernel(const int* __restrict__ count, int n, int* __restrict__ out) {
  if (threadIdx.x == 0) *out = *count > 0 ? n : 0;
}

hipError_t launch_page_gate(const int* count, int n, int* out, hipStream_t st) {
  hipLaunchKernelGGL(page_gate_kernel, dim3(1), dim3(64), 0, st, count, n, out);
  return hipGetLastError();
}

// faiss's inner-product rule over a member query's concatenated pages (one
// thread per query; scores turned into keys in place, the rule, back).
__global__ __launch_bounds__(64) void page_rule_kernel(float* __restrict__ Dacc,
                                                       int64_t* __restrict__ Iacc, int64_t KA,
                                                       int n, int64_t k,
                                                       const int* __restrict__ member) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= n || !member[q]) return;
  float* d = Dacc + (int64_t)q * KA;
  int64_t* i = Iacc + (int64_t)q * KA;
  int64_t nv = 0;
  while (nv < KA && i[nv] >= 0) ++nv;
  if (nv == 0) return;
  for (int64_t j = 0; j < nv; ++j) d[j] = -d[j];
  faiss_ip_tie_order<int64_t>(d, i, (int)nv, (int)k);
  for (int64_t j = 0; j < nv; ++j) d[j] = -d[j];
}

// The k outputs of every member query (grid: n x ceil(k / 256)); entries past
// the pages are empty (k > the rows there are).
__global__ __launch_bounds__(256) void page_emit_kernel(
    int mode, const float* __restrict__ Dacc, const int64_t* __restrict__ Iacc, int64_t KA,
    int64_t k, int rule, const int* __restrict__ member, int64_t id_base, float min_score,
    float* __restrict__ D, int64_t* __restrict__ I) {
  const int q = blockIdx.x;
  const int64_t j = (int64_t)blockIdx.y * 256 + threadIdx.x;
  if (!member[q] || j >= k) return;
  const int64_t id = j < KA ? Iacc[(int64_t)q * KA + j] : -1;
  const float s = id >= 0 ? Dacc[(int64_t)q * KA + j] : 0.0f;
  const bool l2 = mode == MODE_L2 || mode == MODE_L2D;
  emit_result(mode, l2 ? s : -s, id, id_base, min_score, D + (int64_t)q * k + j,
              I + (int64_t)q * k + j);
}

hipError_t launch_page_finish(int mode, float* Dacc, int64_t* Iacc, int64_t KA, int n, int64_t k,
                              int rule, const int* member, int64_t id_base, float min_score,
                              float* D, int64_t* I, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (k < 1 || KA % 64 != 0 || (k + 255) / 256 > 65535) return hipErrorInvalidValue;
  // the inner-product rule itself, where the pages passed over a run of k-th key
  // ties, runs over the first 2k - 1 entries only, as faiss_ip_tie_order reads them
  if (rule) {
    hipLaunchKernelGGL(page_rule_kernel, dim3((n + 63) / 64), dim3(64), 0, st, Dacc, Iacc, KA, n, k,
                       member);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(page_emit_kernel, dim3(n, (unsigned)((k + 255) / 256)), dim3(256), 0, st, mode,
                     Dacc, Iacc, KA, k, rule, member, id_base, min_score, D, I);
  return hipGetLastError();
}

// Shard merge beyond one 64-entry list (k > 64, or inner product's 2k - 1 > 64):
// each part is a raw lexicographic list of k_in entries; one thread per query
// merges the parts' heads (nparts <= 64) into its `need` best entries in
// scratch (sk/si [nq][need]), then faiss's rule (inner product) and the k outputs.
__global__ __launch_bounds__(64) void merge_parts_big_kernel(
    const float* __restrict__ Dp, const int64_t* __restrict__ Ip, int nparts, int nq, int64_t k_in,
    int64_t need, int64_t k, int asc, float* __restrict__ sk, int64_t* __restrict__ si,
    float* __restrict__ D, int64_t* __restrict__ I) {
  __shared__ int64_t heads[64 * 64];
  const int q = blockIdx.x * 64 + threadIdx.x;
  if (q >= nq) return;
  int64_t* head = heads + threadIdx.x * 64;
  for (int p = 0; p < nparts; ++p) head[p] = 0;
  float* ok = sk + (int64_t)q * need;
  int64_t* oi = si + (int64_t)q * need;
  int64_t n = 0;
  for (; n < need; ++n) {
    float bk = FLT_MAX;
    int64_t bi = -1;
    int bp = -1;
    for (int p = 0; p < nparts; ++p) {
      if (head[p] >= k_in) continue;
      const int64_t off = ((int64_t)p * nq + q) * k_in + head[p];
      const int64_t id = Ip[off];
      if (id < 0) {
        head[p] = k_in;  // a raw list ends at its first empty entry
        continue;
      }
      const float key = asc ? Dp[off] : -Dp[off];
      if (bp < 0 || lex_less(key, id, bk, bi)) {
        bk = key;
        bi = id;
        bp = p;
      }
    }
    if (bp < 0) break;
    ++head[bp];
    ok[n] = bk;
    oi[n] = bi;
  }
  for (int64_t j = n; j < need; ++j) {
    ok[j] = FLT_MAX;
    oi[j] = -1;
  }
  if (!asc && n > 0) faiss_ip_tie_order<int64_t>(ok, oi, (int)n, (int)k);
  for (int64_t j = 0; j < k; ++j) {
    const int64_t id = j < need ? oi[j] : -1;
    D[(int64_t)q * k + j] = id >= 0 ? (asc ? ok[j] : -ok[j]) : (asc ? FLT_MAX : -FLT_MAX);
    I[(int64_t)q * k + j] = id;
  }
}

// ---------------------------------------------------------------------------
// Support kernels.
template <typename T>
__global__ __launch_bounds__(256) void row_norms_kernel(const T* __restrict__ X, int64_t ld,
                                                        int64_t r0, int64_t n,
                                                        float* __restrict__ out) {
  constexpr int EPC = 16 / sizeof(T);
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const uint4* xr = (const uint4*)(X + (r0 + row) * ld);
  // fp64 sum of the exact squares, rounded once: |x|^2 correctly rounded to
  // fp32 (up to the fp64 sum's 2^-53-level error), so an L2 key
  // (|q|^2 + |x|^2) - 2 q.x carries only the roundings of its own formula
  // (the strict tie window of oracle/flat.py key_window)
  double s = 0.0;
  for (int64_t c = lane; c < ld / EPC; c += 64) {
    const uint4 v = xr[c];
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (sizeof(T) == 4) {
        const double f = (double)__uint_as_float(u[i]);
        s = fma(f, f, s);
      } else {
        const double a = (double)__uint_as_float(u[i] << 16),
                     b = (double)__uint_as_float(u[i] & 0xFFFF0000u);
        s = fma(a, a, fma(b, b, s));
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) out[r0 + row] = (float)s;
}

hipError_t launch_row_norms(const void* X, int esize, int64_t ld, int64_t r0, int64_t n,
                            float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + 3) / 4;
  if (esize == 4)
    hipLaunchKernelGGL(row_norms_kernel<float>, dim3((unsigned)nb), dim3(256), 0, st,
                       (const float*)X, ld, r0, n, out);
  else
    hipLaunchKernelGGL(row_norms_kernel<uint16_t>, dim3((unsigned)nb), dim3(256), 0, st,
                       (const uint16_t*)X, ld, r0, n, out);
  return hipGetLastError();
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ in, int64_t ldi,
                                   uint16_t* __restrict__ out, int64_t ldo, int64_t rows,
                                   int64_t cols) {
  const int64_t row = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (row >= rows) return;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ldo; j += (int64_t)gridDim.x * 256)
    out[row * ldo + j] = j < cols ? f32_to_bf16_rne(in[row * ldi + j]) : (uint16_t)0;
}

__global__ void bf16_to_f32_kernel(const uint16_t* __restrict__ in, int64_t ldi,
                                   float* __restrict__ out, int64_t ldo, int64_t rows,
                                   int64_t cols) {
  const int64_t row = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (row >= rows) return;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ldo; j += (int64_t)gridDim.x * 256)
    out[row * ldo + j] = j < cols ? __uint_as_float((uint32_t)in[row * ldi + j] << 16) : 0.0f;
}

static dim3 pitched_grid(int64_t rows, int64_t ldo) {
  const int64_t gy = rows < 65535 ? rows : 65535;
  const int64_t gz = (rows + 65534) / 65535;
  const int64_t gx = (ldo + 255) / 256 < 8 ? (ldo + 255) / 256 : 8;
  return dim3((unsigned)gx, (unsigned)gy, (unsigned)gz);
}

// One wave per plane row: 4 elements (8 B) per lane per pass.
__global__ __launch_bounds__(256) void bf16_plane_kernel(const float* __restrict__ X, int64_t ld,
                                                         int64_t r0, int64_t n,
                                                         uint16_t* __restrict__ plane) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const float* xr = X + (r0 + row) * ld;
  char* base = (char*)plane;
  for (int64_t c = lane * 4; c < ld; c += 256) {
    const f32x4 v = *(const f32x4*)(xr + c);
    const uint32_t lo = (uint32_t)f32_to_bf16_rne(v[0]) | ((uint32_t)f32_to_bf16_rne(v[1]) << 16);
    const uint32_t hi = (uint32_t)f32_to_bf16_rne(v[2]) | ((uint32_t)f32_to_bf16_rne(v[3]) << 16);
    *(uint2*)(base + plane_offset(r0 + row, 2 * c, 2 * ld)) = make_uint2(lo, hi);
  }
}

hipError_t launch_bf16_plane(const float* X, int64_t ld, int64_t r0, int64_t n, uint16_t* plane,
                             hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ld % 64 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bf16_plane_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, X, ld, r0,
                     n, plane);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void plane_zero_rows_kernel(char* __restrict__ plane,
                                                              int64_t ldb, int64_t r0, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  for (int64_t c = lane * 16; c < ldb; c += 1024)
    *(uint4*)(plane + plane_offset(r0 + row, c, ldb)) = make_uint4(0, 0, 0, 0);
}

hipError_t launch_plane_zero_rows(char* plane, int64_t ldb, int64_t r0, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (ldb % 64 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(plane_zero_rows_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, plane,
                     ldb, r0, n);
  return hipGetLastError();
}

hipError_t launch_f32_to_bf16(const float* in, int64_t ldi, uint16_t* out, int64_t ldo,
                              int64_t rows, int64_t cols, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(f32_to_bf16_kernel, pitched_grid(rows, ldo), dim3(256), 0, st, in, ldi, out,
                     ldo, rows, cols);
  return hipGetLastError();
}

hipError_t launch_bf16_to_f32(const uint16_t* in, int64_t ldi, float* out, int64_t ldo,
                              int64_t rows, int64_t cols, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(bf16_to_f32_kernel, pitched_grid(rows, ldo), dim3(256), 0, st, in, ldi, out,
                     ldo, rows, cols);
  return hipGetLastError();
}

__global__ void round_bf16_kernel(float* __restrict__ x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = __uint_as_float((uint32_t)f32_to_bf16_rne(x[i]) << 16);
}

hipError_t launch_round_bf16(float* x, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(round_bf16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, n);
  return hipGetLastError();
}

__global__ void rsqrt_kernel(const float* __restrict__ nrm, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (float)(1.0 / sqrt((double)nrm[i]));
}

hipError_t launch_rsqrt(const float* norm, int64_t n, float* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(rsqrt_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, norm, n,
                     out);
  return hipGetLastError();
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__global__ __launch_bounds__(256) void fill_synthetic_kernel(T* __restrict__ out, int64_t rows,
                                                             int64_t d, int64_t ldo, uint64_t seed,
                                                             int64_t row0) {
  const int64_t row = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (row >= rows) return;
  const uint64_t base = (uint64_t)(row0 + row) * (uint64_t)d;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ldo; j += (int64_t)gridDim.x * 256) {
    float v = 0.0f;
    if (j < d) {
      const uint64_t z = splitmix64(seed ^ (base + (uint64_t)j));
      v = (float)(z >> 40) * (1.0f / 8388608.0f) - 1.0f;
    }
    if constexpr (sizeof(T) == 4) out[row * ldo + j] = v;
    else out[row * ldo + j] = f32_to_bf16_rne(v);
  }
}

hipError_t launch_fill_synthetic(void* out, int esize, int64_t rows, int64_t d, int64_t ldo,
                                 uint64_t seed, int64_t row0, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  if (esize == 4)
    hipLaunchKernelGGL(fill_synthetic_kernel<float>, pitched_grid(rows, ldo), dim3(256), 0, st,
                       (float*)out, rows, d, ldo, seed, row0);
  else
    hipLaunchKernelGGL(fill_synthetic_kernel<uint16_t>, pitched_grid(rows, ldo), dim3(256), 0,
                       st, (uint16_t*)out, rows, d, ldo, seed, row0);
  return hipGetLastError();
}

template <typename T>
__global__ __launch_bounds__(256) void fill_synthetic_ids_kernel(T* __restrict__ out,
                                                                 const int64_t* __restrict__ ids,
                                                                 int64_t rows, int64_t d,
                                                                 int64_t ldo, uint64_t seed) {
  const int64_t row = blockIdx.y + (int64_t)blockIdx.z * 65535;
  if (row >= rows) return;
  const uint64_t base = (uint64_t)ids[row] * (uint64_t)d;
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < ldo; j += (int64_t)gridDim.x * 256) {
    float v = 0.0f;
    if (j < d) {
      const uint64_t z = splitmix64(seed ^ (base + (uint64_t)j));
      v = (float)(z >> 40) * (1.0f / 8388608.0f) - 1.0f;
    }
    if constexpr (sizeof(T) == 4) out[row * ldo + j] = v;
    else out[row * ldo + j] = f32_to_bf16_rne(v);
  }
}

hipError_t launch_fill_synthetic_ids(void* out, int esize, const int64_t* ids, int64_t rows,
                                     int64_t d, int64_t ldo, uint64_t seed, hipStream_t st) {
  if (rows <= 0) return hipSuccess;
  if (esize == 4)
    hipLaunchKernelGGL(fill_synthetic_ids_kernel<float>, pitched_grid(rows, ldo), dim3(256), 0,
                       st, (float*)out, ids, rows, d, ldo, seed);
  else
    hipLaunchKernelGGL(fill_synthetic_ids_kernel<uint16_t>, pitched_grid(rows, ldo), dim3(256), 0,
                       st, (uint16_t*)out, ids, rows, d, ldo, seed);
  return hipGetLastError();
}

__global__ void fill_empty_kernel(int asc, float* __restrict__ D, int64_t* __restrict__ I,
                                  int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    D[i] = asc ? FLT_MAX : -FLT_MAX;
    I[i] = -1;
  }
}

hipError_t launch_fill_empty(int mode, float* D, int64_t* I, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_empty_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     (mode == MODE_L2 || mode == MODE_L2D) ? 1 : 0, D, I, n);
  return hipGetLastError();
}

__device__ __forceinline__ int64_t count_less(const int64_t* a, int64_t n, int64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// The kept rows of [src0, src0+n) packed, in order, into out (and their norms
// into out_norms).  removed holds the sorted removed rows of that range only (a
// slice of the whole list).  One workgroup per 64 consecutive rows: two binary
// searches bound the block's removed entries, which flag their rows in LDS; a
// ballot over the flags gives every kept row its packed position; then each
// wave copies 16 rows, 16 B per lane (no per-row search on the copy's path).
constexpr int kKeptRows = 64;
__global__ __launch_bounds__(256) void gather_kept_kernel(const char* __restrict__ X,
                                                          const float* __restrict__ norms,
                                                          int64_t rowbytes, int64_t src0,
                                                          int64_t n,
                                                          const int64_t* __restrict__ removed,
                                                          int64_t nrem, char* __restrict__ out,
                                                          float* __restrict__ out_norms) {
  __shared__ int64_t bound[2];
  __shared__ int flag[kKeptRows];
  __shared__ int64_t dsts[kKeptRows];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kKeptRows;
  const int64_t r0 = src0 + i0;
  if (tid < 2) bound[tid] = count_less(removed, nrem, r0 + (tid ? kKeptRows : 0));
  if (tid < kKeptRows) flag[tid] = 0;
  __syncthreads();
  const int64_t lo = bound[0], hi = bound[1];
  for (int64_t j = lo + tid; j < hi; j += blockDim.x) flag[(int)(removed[j] - r0)] = 1;
  __syncthreads();
  if (w == 0) {
    const bool rm = flag[lane] != 0;
    const uint64_t m = __ballot(rm);
    const int below = __popcll(m & ((1ull << lane) - 1ull));
    dsts[lane] = rm || i0 + lane >= n ? -1 : i0 + lane - (lo + below);
  }
  __syncthreads();
  const int64_t nv = rowbytes >> 4;
  for (int r = w; r < kKeptRows; r += 4) {
    const int64_t dst = dsts[r];
    if (dst < 0) continue;  // uniform over the wave
    const uint4* src = (const uint4*)(X + (r0 + r) * rowbytes);
    uint4* dd = (uint4*)(out + dst * rowbytes);
    for (int64_t c = lane; c < nv; c += 64) dd[c] = src[c];
    if (lane == 0) out_norms[dst] = norms[r0 + r];
  }
}

hipError_t launch_gather_kept(const void* X, const float* norms, int64_t rowbytes, int64_t src0,
                              int64_t n, const int64_t* removed, int64_t nrem, void* out,
                              float* out_norms, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_kept_kernel, dim3((unsigned)((n + kKeptRows - 1) / kKeptRows)), dim3(256), 0, st,
                     (const char*)X, norms, rowbytes, src0, n, removed, nrem, (char*)out,
                     out_norms);
  return hipGetLastError();
}

// out[i] = i for i < n, *count = n: a gathered batch that is every query.
__global__ __launch_bounds__(256) void iota_kernel(int* __restrict__ out, int n,
                                                   int* __restrict__ count) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = i;
  if (i == 0) *count = n;
}

hipError_t launch_iota(int* out, int n, int* count, hipStream_t st) {
  if (n <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(iota_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, n, count);
  return hipGetLastError();
}

// Tombstones (vs_api.hip, vs_remove_ids on an index without filter planes):
// the removed rows keep their place until a pack, filled with NaN (fp32
// 0x7FC00000, bf16 0x7FC0) and a NaN norm, so every kernel's strict admission
// (key < last, lex_less) leaves them out, whatever the metric.  One workgroup
// per row.
__global__ __launch_bounds__(256) void fill_nan_rows_kernel(char* __restrict__ X, int64_t rowbytes,
                                                            float* __restrict__ norms, int esize,
                                                            const int64_t* __restrict__ rows,
                                                            float* __restrict__ scale) {
  const int64_t r = rows[blockIdx.x];
  uint32_t* p = (uint32_t*)(X + r * rowbytes);
  const uint32_t v = esize == 2 ? 0x7FC07FC0u : 0x7FC00000u;
  for (int64_t i = threadIdx.x; i < rowbytes / 4; i += 256) p[i] = v;
  if (threadIdx.x == 0) {
    norms[r] = __uint_as_float(0x7FC00000u);
    if (scale) scale[r] = __uint_as_float(0x7FC00000u);
  }
}

hipError_t launch_fill_nan_rows(void* X, int64_t rowbytes, float* norms, int esize,
                                const int64_t* rows, int64_t n, hipStream_t st, float* scale) {
  if (n <= 0) return hipSuccess;
  if (rowbytes % 4 != 0 || n > INT32_MAX) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fill_nan_rows_kernel, dim3((unsigned)n), dim3(256), 0, st, (char*)X, rowbytes,
                     norms, esize, rows, scale);
  return hipGetLastError();
}

// Search output labels of a tombstoned index: a kernel row p (plus id_base)
// becomes faiss's label, its position among the live rows: p minus the dead
// rows below it (binary search in the sorted dead list; p itself is live).
__global__ __launch_bounds__(256) void label_map_kernel(int64_t* __restrict__ I, int64_t n,
                                                        const int64_t* __restrict__ dead,
                                                        int64_t ndead, int64_t id_base) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int64_t v = I[i];
  if (v < 0) return;
  const int64_t p = v - id_base;
  int64_t lo = 0, hi = ndead;  // first dead row >= p
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (dead[mid] < p) lo = mid + 1;
    else hi = mid;
  }
  I[i] = p - lo + id_base;
}

hipError_t launch_label_map(int64_t* I, int64_t n, const int64_t* dead, int64_t ndead,
                            int64_t id_base, hipStream_t st) {
  if (n <= 0 || ndead <= 0) return hipSuccess;
  hipLaunchKernelGGL(label_map_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, I, n,
                     dead, ndead, id_base);
  return hipGetLastError();
}

}  // namespace vs
