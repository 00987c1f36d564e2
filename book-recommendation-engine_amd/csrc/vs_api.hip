// vs_api.hip — the C-ABI of libvsearch.so (declared in include/vsearch.h).
//
// A vs_index is one device's exact flat index: library-owned row storage in HBM
// (fp32 or bf16 elements, stride `ld` elements = a multiple of 128 B, zero
// padding), the squared norms of every row, and ntotal.  It mirrors faiss::IndexFlat (faiss-cpu 1.11.0, not vendored; see
// /root/reference/poetry.lock:866-867): add copies the caller's rows, search
// writes caller-allocated D/I, remove_ids compacts stably.
//
// Concurrency follows faiss's contract (concurrent searches allowed, add/remove
// exclusive): a shared_mutex guards the storage; per-call scratch comes from the
// stream-ordered allocator so concurrent searches on different streams never
// share workspace.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "../../include/vsearch.h"
#include "vs_internal.h"

using namespace vs;

struct vs_index {
  int d = 0;
  int metric = VS_METRIC_L2;
  int dtype = VS_DTYPE_F32;
  int device = 0;
  int esize = 4;         // bytes per stored element (4 fp32, 2 bf16)
  int64_t ld = 0;        // row stride in elements (ld * esize is a multiple of 128)
  int64_t ntotal = 0;
  int64_t capacity = 0;  // rows allocated (multiple of kRowPad, >= ntotal + kBQ)
  int64_t id_base = 0;
  char* codes = nullptr;   // [capacity][ld] elements
  int64_t rowbytes() const { return ld * esize; }
  char* row(int64_t r) const { return codes + r * rowbytes(); }
  float* norms = nullptr;  // [capacity] squared L2 norms
  // fp32 indexes: a copy of the rows in the blocked layout the bf16x3 GEMM
  // streams (vs_gemm_x3.hip), derived lazily from `codes`; valid for rows
  // [0, blocked_rows).  capacity x ld floats.
  float* blocked = nullptr;
  int64_t blocked_rows = 0;
  // fp32 indexes, filter pass from planes (VS_X2F_SRC=planes): the hi/mid bf16
  // planes of the rows in the order of the filter kernel's LDS images
  // (split_rows_kernel); valid for rows [0, planes_rows).  capacity x ld x 2 bf16.
  uint4* planes = nullptr;
  int64_t planes_rows = 0;
  int engine = VS_ENGINE_AUTO;
  // filter-and-verify fallback rate (moving average over large searches) and a
  // probe counter: see the adaptive choice in run_topk
  double x2v_fallback = 0.0;
  int64_t x2v_probe = 0;
  std::mutex x2v_mu;
  std::mutex blocked_mu;
  std::shared_mutex mu;
};

namespace {

constexpr double kX2vMaxFallback = 0.4;  // filter-and-verify: adaptive switch point

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? VS_E_OOM : VS_E_HIP;
}

#define VS_HIP(expr, what)                    \
  do {                                        \
    hipError_t e_ = (expr);                   \
    if (e_ != hipSuccess) return hip_fail(e_, what); \
  } while (0)

// Selects the index's device for the duration of a call, restoring the caller's.
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Stream-ordered scratch allocation, released on scope exit (on the same stream).
struct Scratch {
  hipStream_t st;
  std::vector<void*> ptrs;
  explicit Scratch(hipStream_t s) : st(s) {}
  hipError_t alloc(void** p, size_t bytes) {
    *p = nullptr;
    if (bytes == 0) return hipSuccess;
    hipError_t e = hipMallocAsync(p, bytes, st);
    if (e == hipSuccess) ptrs.push_back(*p);
    return e;
  }
  ~Scratch() {
    for (void* p : ptrs) (void)hipFreeAsync(p, st);
  }
};

// Kernel timer (measurement hook for bench.py; see vs_timer_* in vsearch.h).
std::mutex g_timer_mu;
bool g_timer_on = false;
struct TimedSpan {
  hipEvent_t a, b;
  int dispatches;
};
std::vector<TimedSpan> g_timer_events;

const char* g_timer_kernel = "";
// filter-and-verify statistics (vs_filter_stats)
int64_t g_filter_queries = 0;
int64_t g_filter_fallbacks = 0;
int64_t g_filter_wide = 0;  // flagged queries given to launch_verify_wide

// The wide verification of flagged queries (VS_X2F_WIDE=0 turns it off, for A/B).
bool x2f_wide_enabled() {
  static const bool on = [] {
    const char* e = getenv("VS_X2F_WIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

struct KernelTimer {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  int dispatches = 1;  // kernel launches between the two events
  KernelTimer(hipStream_t s, const char* name) : st(s) {
    {
      std::lock_guard<std::mutex> g(g_timer_mu);
      g_timer_kernel = name;
    }
    std::lock_guard<std::mutex> g(g_timer_mu);
    if (!g_timer_on) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
      a = b = nullptr;
      return;
    }
    (void)hipEventRecord(a, st);
  }
  void stop() {
    if (!a) return;
    (void)hipEventRecord(b, st);
    std::lock_guard<std::mutex> g(g_timer_mu);
    g_timer_events.push_back({a, b, dispatches});
    a = b = nullptr;
  }
};

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

int kp_for(int64_t k) { return k <= 8 ? 8 : k <= 16 ? 16 : k <= 32 ? 32 : 64; }

// Default source of the filter pass (x2f_source): blocked fp32 rows.
constexpr int kX2fDefaultSource = 0;

void drop_blocked(vs_index* idx) {  // both derived copies of the rows
  if (idx->blocked) (void)hipFree(idx->blocked);
  idx->blocked = nullptr;
  idx->blocked_rows = 0;
  if (idx->planes) (void)hipFree(idx->planes);
  idx->planes = nullptr;
  idx->planes_rows = 0;
}

// Makes the hi/mid planes valid for all rows (as ensure_blocked).
bool ensure_planes(vs_index* idx, hipStream_t st) {
  std::lock_guard<std::mutex> g(idx->blocked_mu);
  const size_t bytes = (size_t)idx->capacity * idx->ld * 2 * sizeof(uint16_t);
  if (!idx->planes) {
    if (hipMalloc(&idx->planes, bytes) != hipSuccess) {
      (void)hipGetLastError();
      idx->planes = nullptr;
      return false;
    }
    idx->planes_rows = 0;
    if (hipMemsetAsync(idx->planes, 0, bytes, st) != hipSuccess) return false;
  }
  if (idx->planes_rows < idx->ntotal) {
    if (launch_split_rows((const float*)idx->codes, idx->ld, idx->planes_rows,
                          idx->ntotal - idx->planes_rows, 2, idx->planes, st) != hipSuccess)
      return false;
    idx->planes_rows = idx->ntotal;
  }
  return true;
}

// Source of the filter pass's database operand: 1 = pre-split planes by
// LDS-DMA, 0 = blocked fp32 rows split in the kernel.  VS_X2F_SRC=planes|blocked
// overrides (read per search, so tests and A/B runs can switch it).
int x2f_source() {
  const char* e = getenv("VS_X2F_SRC");
  if (e && strcmp(e, "planes") == 0) return 1;
  if (e && strcmp(e, "blocked") == 0) return 0;
  return kX2fDefaultSource;
}

// Makes the blocked copy valid for all rows (called under the shared lock;
// builds are serialised by blocked_mu).  Returns false when it cannot be
// allocated (the caller then uses the fp32 MFMA kernel).
bool ensure_blocked(vs_index* idx, hipStream_t st) {
  std::lock_guard<std::mutex> g(idx->blocked_mu);
  if (!idx->blocked) {
    if (hipMalloc(&idx->blocked, (size_t)idx->capacity * idx->ld * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      idx->blocked = nullptr;
      return false;
    }
    idx->blocked_rows = 0;
    // padding rows must hold zeros, like the row storage
    if (hipMemsetAsync(idx->blocked, 0, (size_t)idx->capacity * idx->ld * sizeof(float), st) !=
        hipSuccess)
      return false;
  }
  if (idx->blocked_rows < idx->ntotal) {
    if (launch_block_rows((const float*)idx->codes, idx->ld, idx->blocked_rows,
                          idx->ntotal - idx->blocked_rows, idx->blocked, st) != hipSuccess)
      return false;
    idx->blocked_rows = idx->ntotal;
  }
  return true;
}

int engine_from_env() {
  const char* e = getenv("VS_ENGINE");
  if (!e) return VS_ENGINE_AUTO;
  if (strcmp(e, "fp32") == 0) return VS_ENGINE_FP32_MFMA;
  if (strcmp(e, "bf16x3") == 0) return VS_ENGINE_BF16X3;
  if (strcmp(e, "bf16x2v") == 0) return VS_ENGINE_BF16X2_VERIFY;
  return VS_ENGINE_AUTO;
}

// Grows storage to hold `rows` rows (plus the tile slack), preserving content.
int ensure_capacity(vs_index* idx, int64_t rows, hipStream_t st) {
  const int64_t need = round_up(rows + kBQ, kRowPad);
  if (need <= idx->capacity) return VS_OK;
  int64_t cap = std::max(need, round_up(idx->capacity + idx->capacity / 2, kRowPad));
  char* codes = nullptr;
  float* norms = nullptr;
  hipError_t e = hipMalloc(&codes, (size_t)cap * idx->rowbytes());
  if (e != hipSuccess) {
    // retry without the growth headroom
    cap = need;
    e = hipMalloc(&codes, (size_t)cap * idx->rowbytes());
    if (e != hipSuccess) return hip_fail(e, "vs: allocating row storage");
  }
  e = hipMalloc(&norms, (size_t)cap * sizeof(float));
  if (e != hipSuccess) {
    (void)hipFree(codes);
    return hip_fail(e, "vs: allocating norm storage");
  }
  // zero the whole tail (tile reads past ntotal must see zeros, never NaN garbage)
  const int64_t keep = idx->ntotal;
  VS_HIP(hipMemsetAsync(codes + keep * idx->rowbytes(), 0, (size_t)(cap - keep) * idx->rowbytes(),
                        st),
         "vs: zeroing storage");
  VS_HIP(hipMemsetAsync(norms + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
         "vs: zeroing norms");
  if (idx->codes && keep > 0) {
    VS_HIP(hipMemcpyAsync(codes, idx->codes, (size_t)keep * idx->rowbytes(),
                          hipMemcpyDeviceToDevice, st),
           "vs: copying storage");
    VS_HIP(hipMemcpyAsync(norms, idx->norms, (size_t)keep * sizeof(float),
                          hipMemcpyDeviceToDevice, st),
           "vs: copying norms");
  }
  // In-flight searches (any stream) may still read the old storage.
  VS_HIP(hipDeviceSynchronize(), "vs: storage growth");
  drop_blocked(idx);  // rebuilt lazily at the new capacity
  if (idx->codes) (void)hipFree(idx->codes);
  if (idx->norms) (void)hipFree(idx->norms);
  idx->codes = codes;
  idx->norms = norms;
  idx->capacity = cap;
  return VS_OK;
}

int run_topk(vs_index* idx, int mode, const float* qbuf, const void* qb16, const float* qaux,
             int nq, int nq_pad, int k, int64_t self0, float min_score, float* D, int64_t* I,
             hipStream_t st, const float* xaux, int force_engine, int raw);

// The filter-and-verify engine (vs_gemm_x3.hip): an NP = 2 pass keeps the KF
// best approximate candidates of every query, verify_rescore_kernel proves the
// exact top-`need` is among them (or flags the query), rescores them exactly and
// the usual merge emits (D, I).  Flagged queries are redone by the exact engine.
int run_filter_verify(vs_index* idx, int mode, const float* qbuf, const float* qaux, int nq,
                      int nq_pad, int k, int need, int KF, float min_score, float* D, int64_t* I,
                      hipStream_t st, const float* xaux, int xd, int64_t self0, int raw,
                      int level = 0) {
  const int ntotal = (int)idx->ntotal;
  Scratch scr(st);
  X3Args a;
  a.nq_pad = (int)round_up(nq_pad, kX3Q);
  const int nqt = a.nq_pad / kX3Q;
  const int ntiles = (ntotal + kX3Q - 1) / kX3Q;
  const int L = x2f_lane_len();  // lane list length (<= KF)
  // enough lists that their 2*nsplit*L entries cover 4*KF candidates (KF = 64:
  // eight database splits even when the query tiles alone fill the chip), so the
  // list floors sit well behind the KF-th candidate for the wide check
  a.nsplit = (int)std::max<int64_t>(std::min<int64_t>(ntiles, (2 * KF + L - 1) / L),
                                    std::min<int64_t>(ntiles, (256 + nqt - 1) / nqt));
  a.nsplit = std::max(a.nsplit, 1);
  Partials part;
  part.KP = kp_for(KF);  // lists padded past L, so the merge can emit KF
  part.P = 2 * a.nsplit;
  const size_t np_ = (size_t)a.nq_pad * part.P * part.KP;
  VS_HIP(scr.alloc((void**)&part.key, np_ * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&part.id, np_ * sizeof(int)), "vs: scratch");
  uint4* qp = nullptr;
  const size_t qpb = (size_t)2 * a.nq_pad * idx->ld * sizeof(uint16_t);
  VS_HIP(scr.alloc((void**)&qp, qpb), "vs: scratch");
  if (a.nq_pad > nq_pad) VS_HIP(hipMemsetAsync(qp, 0, qpb, st), "vs: query planes");
  VS_HIP(launch_split_queries(qbuf, idx->ld, nq_pad, a.nq_pad, 2, qp, st), "vs: query planes");
  // |q|^2 (L2 searches stage it in qaux already) and max |x|^2 for the bound
  const float* qn = qaux;
  if (mode != MODE_L2) {
    float* t = nullptr;
    VS_HIP(scr.alloc((void**)&t, (size_t)nq_pad * sizeof(float)), "vs: scratch");
    VS_HIP(launch_row_norms(qbuf, 4, idx->ld, 0, nq_pad, t, st), "vs: query norms");
    qn = t;
  }
  unsigned* xmax2 = nullptr;
  VS_HIP(scr.alloc((void**)&xmax2, sizeof(unsigned)), "vs: scratch");
  VS_HIP(launch_max_norm(idx->norms, ntotal, xmax2, st), "vs: max norm");
  a.XB = xd ? (const float*)idx->planes : idx->blocked;
  a.xaux = xaux;
  a.QP = qp;
  a.qaux = qaux;
  a.nqa = nq_pad;
  a.ld = idx->ld;
  a.ntotal = ntotal;
  a.self0 = self0;  // self-join: query q is row self0 + q, never its own candidate
  {
    KernelTimer tm(st, "gemm_topk_x2f");
    VS_HIP(launch_gemm_topk_x3(L, mode, 2, xd, a, part, st, &tm.dispatches),
           "vs: gemm_topk_x2f launch");
    tm.stop();
  }
  // approximate top-KF per query (plain lexicographic order: the L2 merge)
  float* Dk = nullptr;
  int64_t* Ik = nullptr;
  VS_HIP(scr.alloc((void**)&Dk, (size_t)nq * KF * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&Ik, (size_t)nq * KF * sizeof(int64_t)), "vs: scratch");
  VS_HIP(launch_merge_partials(MODE_L2, part, nq, KF, 0, 0.0f, Dk, Ik, KF, st), "vs: merge");
  Partials vp;
  vp.KP = kp_for(KF);
  vp.P = 1;
  int* fail_d = nullptr;
  VS_HIP(scr.alloc((void**)&vp.key, (size_t)nq * vp.KP * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&vp.id, (size_t)nq * vp.KP * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&fail_d, (size_t)nq * sizeof(int)), "vs: scratch");
  // cosine (self-join): qaux / xaux are the inverse norms the keys are scaled by
  const double coef = mode == MODE_COS ? x2f_cos_key_bound(idx->ld) : x2f_bound_coef(idx->ld);
  VS_HIP(launch_verify_rescore(mode, nq, KF, need, Dk, Ik, (const float*)idx->codes, idx->norms,
                               qbuf, qn, idx->ld, coef, xmax2, part, L, vp.key, vp.id, vp.KP,
                               fail_d, st, mode == MODE_COS ? qaux : nullptr,
                               mode == MODE_COS ? xaux : nullptr),
         "vs: verify");
  // queries the bound could not settle on KF candidates: rescore every lane-list
  // entry below the list floors (launch_verify_wide), then the rest go on below
  std::vector<int> fh(nq);
  VS_HIP(hipMemcpyAsync(fh.data(), fail_d, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st),
         "vs: verify flags");
  VS_HIP(hipStreamSynchronize(st), "vs: verify flags");
  std::vector<int> F;
  for (int q = 0; q < nq; ++q)
    if (fh[q]) F.push_back(q);
  if (!F.empty() && x2f_wide_enabled()) {
    int* qlist = nullptr;
    VS_HIP(scr.alloc((void**)&qlist, F.size() * sizeof(int)), "vs: scratch");
    VS_HIP(hipMemcpyAsync(qlist, F.data(), F.size() * sizeof(int), hipMemcpyHostToDevice, st),
           "vs: verify list");
    VS_HIP(launch_verify_wide(mode, (int)F.size(), qlist, KF, need, (const float*)idx->codes,
                              idx->norms, qbuf, qn, idx->ld, coef, xmax2, part, L, vp.key, vp.id,
                              vp.KP, fail_d, st, mode == MODE_COS ? qaux : nullptr,
                              mode == MODE_COS ? xaux : nullptr),
           "vs: verify wide");
    VS_HIP(hipMemcpyAsync(fh.data(), fail_d, (size_t)nq * sizeof(int), hipMemcpyDeviceToHost, st),
           "vs: verify flags");
    VS_HIP(hipStreamSynchronize(st), "vs: verify flags");  // qlist's copy is done too
    {
      std::lock_guard<std::mutex> g(g_timer_mu);
      g_filter_wide += (int64_t)F.size();
    }
    F.clear();
    for (int q = 0; q < nq; ++q)
      if (fh[q]) F.push_back(q);
  }
  VS_HIP(launch_merge_partials(mode, vp, nq, k, idx->id_base, min_score, D, I, k, st, raw),
         "vs: merge");
  const int nf = (int)F.size();
  // More than 32 flagged queries (and room for more candidates): a second filter
  // pass over just those, keeping 64 candidates, settles most of them for about
  // 1/16 of a full pass per 256 queries; what it cannot settle goes to the exact
  // engine.  The stats count queries that reach the exact engine.
  const bool second = level == 0 && self0 < 0 && KF < 64 && x2f_list_len(need) > 0 &&
                      need + 8 <= 64 && nf > 32;
  {
    std::lock_guard<std::mutex> g(g_timer_mu);
    if (level == 0) g_filter_queries += nq;
    if (!second) g_filter_fallbacks += nf;
  }
  if (level == 0) {
    std::lock_guard<std::mutex> g(idx->x2v_mu);
    const double w = std::min(1.0, nq / 1024.0) * 0.5;  // small batches move it less
    idx->x2v_fallback = (1.0 - w) * idx->x2v_fallback + w * ((double)nf / nq);
  }
  if (F.empty()) return VS_OK;
  // self-joins: the flagged queries are not consecutive rows, so they are redone
  // as plain searches for k + 1 and their own row is dropped afterwards
  const int kf = self0 >= 0 ? k + 1 : k;
  const int nf_pad = (int)round_up(std::max(nf, kGemvMaxQ), kBQ) + kBQ;  // chunk tails
  float* q2 = nullptr;
  float* a2 = nullptr;
  float* D2 = nullptr;
  int64_t* I2 = nullptr;
  VS_HIP(scr.alloc((void**)&q2, (size_t)nf_pad * idx->ld * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&a2, (size_t)nf_pad * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&D2, (size_t)nf * kf * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&I2, (size_t)nf * kf * sizeof(int64_t)), "vs: scratch");
  VS_HIP(hipMemsetAsync(q2, 0, (size_t)nf_pad * idx->ld * sizeof(float), st), "vs: fallback");
  VS_HIP(hipMemsetAsync(a2, 0, (size_t)nf_pad * sizeof(float), st), "vs: fallback");
  for (int i = 0; i < nf; ++i) {
    VS_HIP(hipMemcpyAsync(q2 + (int64_t)i * idx->ld, qbuf + (int64_t)F[i] * idx->ld,
                          (size_t)idx->ld * sizeof(float), hipMemcpyDeviceToDevice, st),
           "vs: fallback");
    if (mode == MODE_L2 || mode == MODE_COS)  // |q|^2, or 1/|q| for cosine
      VS_HIP(hipMemcpyAsync(a2 + i, qaux + F[i], sizeof(float), hipMemcpyDeviceToDevice, st),
             "vs: fallback");
  }
  if (second) {
    int rc = run_filter_verify(idx, mode, q2, a2, nf, nf_pad, k, need, 64, min_score, D2, I2, st,
                               xaux, xd, -1, raw, 1);
    if (rc) return rc;
  }
  // a few queries: 16 at a time through the small-batch kernels (one corpus
  // stream each); more: one exact-engine launch
  const int step = nf <= 64 ? 16 : nf;
  for (int f0 = 0; f0 < (second ? 0 : nf); f0 += step) {
    const int nc = std::min(step, nf - f0);
    const int nc_pad = (int)round_up(std::max(nc, kGemvMaxQ), kBQ);
    int rc = run_topk(idx, mode, q2 + (int64_t)f0 * idx->ld, nullptr, a2 + f0, nc, nc_pad, kf, -1,
                      min_score, D2 + (int64_t)f0 * kf, I2 + (int64_t)f0 * kf, st, xaux,
                      VS_ENGINE_BF16X3, raw);
    if (rc) return rc;
  }
  {
    std::lock_guard<std::mutex> g(g_timer_mu);
    g_timer_kernel = "gemm_topk_x2f";  // the fallback is part of this engine's search
  }
  if (self0 >= 0) {  // drop each query's own row (first occurrence), keep k entries
    std::vector<float> dh((size_t)nf * kf), dk((size_t)nf * k);
    std::vector<int64_t> ih((size_t)nf * kf), ik((size_t)nf * k);
    VS_HIP(hipMemcpyAsync(dh.data(), D2, dh.size() * sizeof(float), hipMemcpyDeviceToHost, st),
           "vs: fallback");
    VS_HIP(hipMemcpyAsync(ih.data(), I2, ih.size() * sizeof(int64_t), hipMemcpyDeviceToHost, st),
           "vs: fallback");
    VS_HIP(hipStreamSynchronize(st), "vs: fallback");
    for (int i = 0; i < nf; ++i) {
      const int64_t self = idx->id_base + self0 + F[i];
      int o = 0;
      bool dropped = false;
      for (int j = 0; j < kf && o < k; ++j) {
        if (!dropped && ih[(size_t)i * kf + j] == self) {
          dropped = true;
          continue;
        }
        dk[(size_t)i * k + o] = dh[(size_t)i * kf + j];
        ik[(size_t)i * k + o] = ih[(size_t)i * kf + j];
        ++o;
      }
    }
    VS_HIP(hipMemcpyAsync(D2, dk.data(), dk.size() * sizeof(float), hipMemcpyHostToDevice, st),
           "vs: fallback");
    VS_HIP(hipMemcpyAsync(I2, ik.data(), ik.size() * sizeof(int64_t), hipMemcpyHostToDevice, st),
           "vs: fallback");
    VS_HIP(hipStreamSynchronize(st), "vs: fallback");  // dk / ik leave scope
  }
  for (int i = 0; i < nf; ++i) {
    VS_HIP(hipMemcpyAsync(D + (int64_t)F[i] * k, D2 + (int64_t)i * k, (size_t)k * sizeof(float),
                          hipMemcpyDeviceToDevice, st),
           "vs: fallback");
    VS_HIP(hipMemcpyAsync(I + (int64_t)F[i] * k, I2 + (int64_t)i * k, (size_t)k * sizeof(int64_t),
                          hipMemcpyDeviceToDevice, st),
           "vs: fallback");
  }
  return VS_OK;
}

// Shared search driver: queries already staged in `qbuf` ([nq_pad][ld] device,
// zero-padded) with query aux values (`qaux`, L2 norms or 1/|q|).
int run_topk(vs_index* idx, int mode, const float* qbuf, const void* qb16, const float* qaux,
             int nq, int nq_pad, int k, int64_t self0, float min_score, float* D, int64_t* I,
             hipStream_t st, const float* xaux, int force_engine = VS_ENGINE_AUTO,
             int raw = 0) {
  // faiss's inner-product tie rule (vs_support.hip, faiss_ip_tie_order) needs the
  // lowest 2k-1 (key, label) entries of every partial list to be exact; `raw`
  // output (plain lexicographic order) needs k.
  const bool tie_rule = mode == MODE_IP && !raw;
  const int KP = tie_rule ? kp_for(std::min(2 * k - 1, VS_MAX_K)) : kp_for(k);
  const int ntotal = (int)idx->ntotal;
  Scratch scr(st);
  Partials part;
  part.KP = KP;

  // Small batches stream the corpus once: the skinny MFMA kernel (any metric /
  // dtype), except fp32 L2 with nq <= 8, which keeps faiss's direct sum (x-q)^2
  // branch on the GEMV kernel.  VS_SMALL_BATCH=gemv|skinny overrides (A/B runs).
  static const char* pref = getenv("VS_SMALL_BATCH");
  const bool small_ok = (mode == MODE_IP || mode == MODE_L2) && self0 < 0;
  const bool gemv_ok = small_ok && nq <= kGemvMaxQ &&
                       (size_t)kGemvMaxQ * idx->ld * sizeof(float) + 4 * kGemvMaxQ * 64 * 8 <=
                           64 * 1024;
  const bool skinny_ok = small_ok && nq <= kSkinnyMaxQ && KP <= 32 && (nq <= 16 || KP <= 16) &&
                         (idx->ld * idx->esize) % 64 == 0;
  bool gemv;
  bool skinny;
  if (pref && strcmp(pref, "gemv") == 0) {
    gemv = gemv_ok;
    skinny = !gemv && skinny_ok;
  } else if (pref && strcmp(pref, "skinny") == 0) {
    skinny = skinny_ok;
    gemv = !skinny && gemv_ok;
  } else {
    // measured (MI355X, 10M x 1536): fp32 batch-1 GEMV 83 % of HBM vs skinny 76 %;
    // bf16 batch-8 skinny 80 % vs GEMV 29 % (profiles/r01_small_batch_ab.txt)
    gemv = gemv_ok && idx->esize == 4 && (nq <= 2 || mode == MODE_L2);
    skinny = !gemv && skinny_ok;
  }
  if (skinny) {
    const int nblocks =
        (int)std::min<int64_t>(2048, std::max<int64_t>(1, (idx->ntotal + 255) / 256));
    part.P = nblocks;
    const size_t n = (size_t)nq * part.P * KP;
    VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
    const void* qsk = qb16 ? qb16 : (const void*)qbuf;
    KernelTimer tm(st, "skinny_topk");
    VS_HIP(launch_skinny_topk(KP, mode, nq, idx->codes, idx->esize, xaux, qsk, qaux, idx->ld,
                              ntotal, nblocks, part, st),
           "vs: skinny_topk launch");
    tm.stop();
    VS_HIP(launch_merge_partials(mode, part, nq, k, idx->id_base, min_score, D, I, k, st, raw),
           "vs: merge launch");
    return VS_OK;
  }
  // bf16 indexes hand the GEMM a bf16 copy of the (already rounded) queries
  const void* qmat = qb16 ? qb16 : (const void*)qbuf;
  if (gemv) {
    const int gmode = mode == MODE_L2 ? MODE_L2D : MODE_IP;
    int nblocks = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (idx->ntotal + 255) / 256));
    part.P = nblocks;
    const int nql = nq <= 2 ? nq : (nq <= 4 ? 4 : 8);
    const size_t n = (size_t)nql * part.P * KP;
    VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
    KernelTimer tm(st, "gemv_topk");
    VS_HIP(launch_gemv_topk(KP, gmode, nq, idx->codes, idx->esize, qbuf, idx->ld, ntotal, nblocks,
                            part, st),
           "vs: gemv_topk launch");
    tm.stop();
    VS_HIP(launch_merge_partials(gmode, part, nq, k, idx->id_base, min_score, D, I, k, st, raw),
           "vs: merge launch");
    return VS_OK;
  }

  // fp32 indexes run the large-batch GEMM on the bf16 matrix cores through the
  // exact 3-plane split (vs_gemm_x3.hip) unless disabled (VS_ENGINE=fp32 /
  // vs_set_engine) or the blocked copy of the rows does not fit in HBM.
  int engine = force_engine != VS_ENGINE_AUTO ? force_engine
               : idx->engine != VS_ENGINE_AUTO ? idx->engine
                                               : engine_from_env();
  // entries of each partial list the final merge needs (faiss's IP tie rule: 2k-1)
  const int need = tie_rule ? std::min(2 * k - 1, VS_MAX_K) : k;
  const int KF = x2f_list_len(need);
  const bool library_choice = engine == VS_ENGINE_AUTO;
  if (engine == VS_ENGINE_AUTO) engine = KF > 0 ? VS_ENGINE_BF16X2_VERIFY : VS_ENGINE_BF16X3;
  // the filter pass: IP / L2 searches, and cosine self-joins from blocked rows
  if (engine == VS_ENGINE_BF16X2_VERIFY &&
      (KF == 0 || (mode == MODE_COS && (self0 < 0 || x2f_source() != 0))))
    engine = VS_ENGINE_BF16X3;
  // Adaptive: a query falls back when its top scores crowd inside the filter's
  // error bound.  The filter pass costs ~0.53 of the exact engine, so once the
  // recent fallback rate passes 0.4 (break-even ~0.47) the exact engine runs
  // directly; every 16th search still takes the filter path to re-measure.
  if (library_choice && engine == VS_ENGINE_BF16X2_VERIFY) {
    std::lock_guard<std::mutex> g(idx->x2v_mu);
    if (idx->x2v_fallback > kX2vMaxFallback && idx->x2v_probe++ % 16 != 0)
      engine = VS_ENGINE_BF16X3;
  }
  if (idx->esize == 4 && engine == VS_ENGINE_BF16X2_VERIFY) {
    const int xd = x2f_source();
    if (xd ? ensure_planes(idx, st) : ensure_blocked(idx, st))
      return run_filter_verify(idx, mode, qbuf, qaux, nq, nq_pad, k, need, KF, min_score, D, I,
                               st, xaux, xd, self0, raw);
  }
  const int KR = x3_list_len(need);
  if (idx->esize == 4 && engine == VS_ENGINE_BF16X3 && KR > 0 && ensure_blocked(idx, st)) {
    X3Args a;
    a.nq_pad = (int)round_up(nq_pad, kX3Q);
    const int nqt3 = a.nq_pad / kX3Q;
    const int ntiles3 = (ntotal + kX3Q - 1) / kX3Q;
    // one 8-wave workgroup per CU on 256 CUs
    a.nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles3, (256 + nqt3 - 1) / nqt3));
    part.P = 2 * a.nsplit;
    const size_t n3 = (size_t)a.nq_pad * part.P * KP;
    VS_HIP(scr.alloc((void**)&part.key, n3 * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, n3 * sizeof(int)), "vs: scratch");
    // query planes (self-join queries are stored rows, split the same way);
    // rows past nq_pad stay zero
    uint4* qp = nullptr;
    const size_t qpb = (size_t)3 * a.nq_pad * idx->ld * sizeof(uint16_t);
    VS_HIP(scr.alloc((void**)&qp, qpb), "vs: scratch");
    if (a.nq_pad > nq_pad) VS_HIP(hipMemsetAsync(qp, 0, qpb, st), "vs: query planes");
    VS_HIP(launch_split_queries(qbuf, idx->ld, nq_pad, a.nq_pad, 3, qp, st), "vs: query planes");
    a.XB = idx->blocked;
    a.xaux = xaux;
    a.QP = qp;
    a.qaux = qaux;
    a.nqa = nq_pad;
    a.ld = idx->ld;
    a.ntotal = ntotal;
    a.self0 = self0;
    KernelTimer tm(st, "gemm_topk_x3");
    VS_HIP(launch_gemm_topk_x3(KR, mode, 3, 0, a, part, st, &tm.dispatches),
           "vs: gemm_topk_x3 launch");
    tm.stop();
    VS_HIP(launch_merge_partials(mode, part, nq, k, idx->id_base, min_score, D, I, k, st, raw),
           "vs: merge launch");
    return VS_OK;
  }

  const int nqt = nq_pad / kBQ;
  const int ntiles = (ntotal + kBN - 1) / kBN;
  // ~2 workgroups per CU on 256 CUs; never more splits than database tiles.
  int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, (512 + nqt - 1) / nqt));
  part.P = 2 * nsplit;
  const size_t n = (size_t)nq_pad * part.P * KP;
  VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
  KernelTimer tm(st, "gemm_topk");
  VS_HIP(launch_gemm_topk(KP, mode, idx->codes, xaux, qmat, qaux, idx->ld, idx->esize, ntotal,
                          nq_pad, nsplit, self0, part, st),
         "vs: gemm_topk launch");
  tm.stop();
  VS_HIP(launch_merge_partials(mode, part, nq, k, idx->id_base, min_score, D, I, k, st, raw),
         "vs: merge launch");
  return VS_OK;
}

}  // namespace

extern "C" {

const char* vs_last_error(void) { return g_err.c_str(); }

int vs_version(void) { return 100; }

int vs_device_count(int* n) {
  if (!n) return fail(VS_E_INVALID, "vs_device_count: null output");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *n = 0;
    return hip_fail(e, "vs_device_count");
  }
  *n = c;
  return VS_OK;
}

int vs_create(int d, int metric, int dtype, int device, vs_index** out) {
  if (!out) return fail(VS_E_INVALID, "vs_create: null output");
  *out = nullptr;
  if (d <= 0) return fail(VS_E_INVALID, "vs_create: d must be > 0");
  if (metric != VS_METRIC_L2 && metric != VS_METRIC_INNER_PRODUCT)
    return fail(VS_E_INVALID, "vs_create: metric must be METRIC_L2 or METRIC_INNER_PRODUCT");
  if (dtype != VS_DTYPE_F32 && dtype != VS_DTYPE_BF16)
    return fail(VS_E_INVALID, "vs_create: dtype must be VS_DTYPE_F32 or VS_DTYPE_BF16");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) return fail(VS_E_HIP, "vs_create: no HIP device available");
  if (device < 0 || device >= ndev) return fail(VS_E_INVALID, "vs_create: bad device ordinal");
  DeviceGuard g(device);
  if (!g.ok) return fail(VS_E_HIP, "vs_create: hipSetDevice failed");
  // Keep freed stream-ordered scratch cached in the pool instead of returning it
  // to the driver at every synchronisation.
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
    uint64_t thr = UINT64_MAX;
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  vs_index* idx = new vs_index();
  idx->d = d;
  idx->metric = metric;
  idx->dtype = dtype;
  idx->device = device;
  idx->esize = dtype == VS_DTYPE_BF16 ? 2 : 4;
  idx->ld = round_up(d, 128 / idx->esize);  // 128-B rows per GEMM stage
  *out = idx;
  return VS_OK;
}

int vs_destroy(vs_index* idx) {
  if (!idx) return VS_OK;
  {
    DeviceGuard g(idx->device);
    (void)hipDeviceSynchronize();
    drop_blocked(idx);
    if (idx->codes) (void)hipFree(idx->codes);
    if (idx->norms) (void)hipFree(idx->norms);
  }
  delete idx;
  return VS_OK;
}

int vs_reserve(vs_index* idx, int64_t n) {
  if (!idx) return fail(VS_E_INVALID, "vs_reserve: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_reserve: n < 0");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  return ensure_capacity(idx, std::max(n, idx->ntotal), nullptr);
}

int vs_add(vs_index* idx, const float* x, int64_t n, int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_add: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_add: n < 0");
  if (n == 0) return VS_OK;
  if (!x) return fail(VS_E_INVALID, "vs_add: null vectors");
  if (idx->ntotal + n >= (int64_t)INT32_MAX - 2 * kRowPad)
    return fail(VS_E_UNSUPPORTED, "vs_add: a shard holds fewer than 2^31 rows");
  hipStream_t st = (hipStream_t)stream;
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  int rc = ensure_capacity(idx, idx->ntotal + n, st);
  if (rc) return rc;
  const hipMemcpyKind kind = (flags & VS_IN_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (idx->esize == 4) {
    VS_HIP(hipMemcpy2DAsync(idx->row(idx->ntotal), idx->rowbytes(), x,
                            (size_t)idx->d * sizeof(float), (size_t)idx->d * sizeof(float),
                            (size_t)n, kind, st),
           "vs_add: copying rows");
  } else {
    // bf16 storage: stage fp32 rows on the device in bounded chunks, round into place
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64ull << 20) / (idx->d * 4));
    Scratch scr(st);
    float* tmp = nullptr;
    VS_HIP(scr.alloc((void**)&tmp, (size_t)std::min(chunk, n) * idx->d * sizeof(float)),
           "vs_add: scratch");
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
      const int64_t m = std::min(chunk, n - r0);
      VS_HIP(hipMemcpyAsync(tmp, x + r0 * idx->d, (size_t)m * idx->d * sizeof(float), kind, st),
             "vs_add: staging rows");
      VS_HIP(launch_f32_to_bf16(tmp, idx->d, (uint16_t*)idx->row(idx->ntotal + r0), idx->ld, m,
                                idx->d, st),
             "vs_add: rounding to bf16");
    }
    VS_HIP(hipStreamSynchronize(st), "vs_add: synchronise");
  }
  VS_HIP(launch_row_norms(idx->codes, idx->esize, idx->ld, idx->ntotal, n, idx->norms, st),
         "vs_add: norms");
  // Source host buffers may be released by the caller as soon as we return.
  VS_HIP(hipStreamSynchronize(st), "vs_add: synchronise");
  idx->ntotal += n;
  return VS_OK;
}

int vs_add_synthetic(vs_index* idx, int64_t n, uint64_t seed, int64_t row0, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_add_synthetic: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_add_synthetic: n < 0");
  if (n == 0) return VS_OK;
  if (idx->ntotal + n >= (int64_t)INT32_MAX - 2 * kRowPad)
    return fail(VS_E_UNSUPPORTED, "vs_add_synthetic: a shard holds fewer than 2^31 rows");
  hipStream_t st = (hipStream_t)stream;
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  int rc = ensure_capacity(idx, idx->ntotal + n, st);
  if (rc) return rc;
  VS_HIP(launch_fill_synthetic(idx->row(idx->ntotal), idx->esize, n, idx->d, idx->ld, seed, row0,
                               st),
         "vs_add_synthetic: fill");
  VS_HIP(launch_row_norms(idx->codes, idx->esize, idx->ld, idx->ntotal, n, idx->norms, st),
         "vs_add_synthetic: norms");
  VS_HIP(hipStreamSynchronize(st), "vs_add_synthetic: synchronise");
  idx->ntotal += n;
  return VS_OK;
}

int vs_add_synthetic_ids(vs_index* idx, const int64_t* ids, int64_t n, uint64_t seed,
                         void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_add_synthetic_ids: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_add_synthetic_ids: n < 0");
  if (n == 0) return VS_OK;
  if (!ids) return fail(VS_E_INVALID, "vs_add_synthetic_ids: null ids");
  if (idx->ntotal + n >= (int64_t)INT32_MAX - 2 * kRowPad)
    return fail(VS_E_UNSUPPORTED, "vs_add_synthetic_ids: a shard holds fewer than 2^31 rows");
  hipStream_t st = (hipStream_t)stream;
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  int rc = ensure_capacity(idx, idx->ntotal + n, st);
  if (rc) return rc;
  Scratch scr(st);
  int64_t* dids = nullptr;
  VS_HIP(scr.alloc((void**)&dids, (size_t)n * sizeof(int64_t)), "vs_add_synthetic_ids: scratch");
  VS_HIP(hipMemcpyAsync(dids, ids, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice, st),
         "vs_add_synthetic_ids: upload");
  VS_HIP(launch_fill_synthetic_ids(idx->row(idx->ntotal), idx->esize, dids, n, idx->d, idx->ld,
                                   seed, st),
         "vs_add_synthetic_ids: fill");
  VS_HIP(launch_row_norms(idx->codes, idx->esize, idx->ld, idx->ntotal, n, idx->norms, st),
         "vs_add_synthetic_ids: norms");
  VS_HIP(hipStreamSynchronize(st), "vs_add_synthetic_ids: synchronise");
  idx->ntotal += n;
  return VS_OK;
}

int vs_reset(vs_index* idx) {
  if (!idx) return fail(VS_E_INVALID, "vs_reset: null index");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  VS_HIP(hipDeviceSynchronize(), "vs_reset");
  drop_blocked(idx);
  if (idx->codes) (void)hipFree(idx->codes);
  if (idx->norms) (void)hipFree(idx->norms);
  idx->codes = nullptr;
  idx->norms = nullptr;
  idx->capacity = 0;
  idx->ntotal = 0;
  return VS_OK;
}

int vs_ntotal(const vs_index* idx, int64_t* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_ntotal: null argument");
  *out = idx->ntotal;
  return VS_OK;
}

int vs_dim(const vs_index* idx, int* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_dim: null argument");
  *out = idx->d;
  return VS_OK;
}

int vs_metric(const vs_index* idx, int* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_metric: null argument");
  *out = idx->metric;
  return VS_OK;
}

int vs_dtype(const vs_index* idx, int* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_dtype: null argument");
  *out = idx->dtype;
  return VS_OK;
}

int vs_set_engine(vs_index* idx, int engine) {
  if (!idx) return fail(VS_E_INVALID, "vs_set_engine: null index");
  if (engine != VS_ENGINE_AUTO && engine != VS_ENGINE_FP32_MFMA && engine != VS_ENGINE_BF16X3 &&
      engine != VS_ENGINE_BF16X2_VERIFY)
    return fail(VS_E_INVALID, "vs_set_engine: unknown engine");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  idx->engine = engine;
  return VS_OK;
}

int vs_set_id_base(vs_index* idx, int64_t id_base) {
  if (!idx) return fail(VS_E_INVALID, "vs_set_id_base: null index");
  if (id_base < 0) return fail(VS_E_INVALID, "vs_set_id_base: negative base");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  idx->id_base = id_base;
  return VS_OK;
}

int vs_search(vs_index* idx, const float* x, int64_t n, int64_t k, float* D, int64_t* I,
              int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_search: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_search: n < 0");
  if (k <= 0) return fail(VS_E_INVALID, "vs_search: k must be > 0");  // faiss: FAISS_THROW_IF_NOT(k > 0)
  if (k > VS_MAX_K) return fail(VS_E_UNSUPPORTED, "vs_search: k > VS_MAX_K (64) not supported yet");
  if (n == 0) return VS_OK;
  if (!x || !D || !I) return fail(VS_E_INVALID, "vs_search: null buffer");
  hipStream_t st = (hipStream_t)stream;
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  if (!g.ok) return fail(VS_E_HIP, "vs_search: hipSetDevice failed");
  const bool out_dev = (flags & VS_OUT_DEVICE) != 0;
  const int mode = idx->metric == VS_METRIC_L2 ? MODE_L2 : MODE_IP;
  Scratch scr(st);

  float* Dd = D;
  int64_t* Id = I;
  if (!out_dev) {
    VS_HIP(scr.alloc((void**)&Dd, (size_t)n * k * sizeof(float)), "vs_search: scratch");
    VS_HIP(scr.alloc((void**)&Id, (size_t)n * k * sizeof(int64_t)), "vs_search: scratch");
  }
  if (idx->ntotal == 0) {
    VS_HIP(launch_fill_empty(mode, Dd, Id, n * k, st), "vs_search: fill");
  } else {
    // Queries are processed in chunks so that scratch stays bounded for any n.
    const int64_t chunk = 65536;
    float* qbuf = nullptr;
    float* qaux = nullptr;
    const int64_t cmax = std::min<int64_t>(n, chunk);
    const int64_t qrows = round_up(std::max<int64_t>(cmax, kGemvMaxQ), kBQ);
    VS_HIP(scr.alloc((void**)&qbuf, (size_t)qrows * idx->ld * sizeof(float)), "vs_search: scratch");
    VS_HIP(scr.alloc((void**)&qaux, (size_t)qrows * sizeof(float)), "vs_search: scratch");
    uint16_t* qb16 = nullptr;
    if (idx->esize == 2)
      VS_HIP(scr.alloc((void**)&qb16, (size_t)qrows * idx->ld * sizeof(uint16_t)),
             "vs_search: scratch");
    const hipMemcpyKind kind =
        (flags & VS_IN_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
    for (int64_t c0 = 0; c0 < n; c0 += chunk) {
      const int64_t nc = std::min(chunk, n - c0);
      const int64_t nq_pad = round_up(std::max<int64_t>(nc, kGemvMaxQ), kBQ);
      // zero what the copy leaves: padding rows, and the column tail when d < ld
      if (idx->d == idx->ld) {
        if (nq_pad > nc)
          VS_HIP(hipMemsetAsync(qbuf + nc * idx->ld, 0,
                                (size_t)(nq_pad - nc) * idx->ld * sizeof(float), st),
                 "vs_search: zero queries");
      } else {
        VS_HIP(hipMemsetAsync(qbuf, 0, (size_t)nq_pad * idx->ld * sizeof(float), st),
               "vs_search: zero queries");
      }
      VS_HIP(hipMemcpy2DAsync(qbuf, idx->ld * sizeof(float), x + c0 * idx->d,
                              (size_t)idx->d * sizeof(float), (size_t)idx->d * sizeof(float),
                              (size_t)nc, kind, st),
             "vs_search: staging queries");
      if (idx->esize == 2) {
        // bf16 index: queries are rounded to bf16 too, so every path (GEMV in fp32
        // on the rounded values, GEMM on bf16 operands) scores the same numbers
        VS_HIP(launch_round_bf16(qbuf, nq_pad * idx->ld, st), "vs_search: rounding queries");
        VS_HIP(launch_f32_to_bf16(qbuf, idx->ld, qb16, idx->ld, nq_pad, idx->ld, st),
               "vs_search: bf16 queries");
      }
      if (mode == MODE_L2)
        VS_HIP(launch_row_norms(qbuf, 4, idx->ld, 0, nq_pad, qaux, st), "vs_search: query norms");
      int rc = run_topk(idx, mode, qbuf, qb16, qaux, (int)nc, (int)nq_pad, (int)k, -1, 0.0f,
                        Dd + c0 * k, Id + c0 * k, st, idx->norms, VS_ENGINE_AUTO,
                        (flags & VS_RAW_ORDER) ? 1 : 0);
      if (rc) return rc;
    }
  }
  if (!out_dev) {
    VS_HIP(hipMemcpyAsync(D, Dd, (size_t)n * k * sizeof(float), hipMemcpyDeviceToHost, st),
           "vs_search: copy D");
    VS_HIP(hipMemcpyAsync(I, Id, (size_t)n * k * sizeof(int64_t), hipMemcpyDeviceToHost, st),
           "vs_search: copy I");
    VS_HIP(hipStreamSynchronize(st), "vs_search: synchronise");
  } else {
    VS_HIP(hipGetLastError(), "vs_search");
  }
  return VS_OK;
}

int vs_reconstruct_n(vs_index* idx, int64_t i0, int64_t n, float* out, int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_reconstruct_n: null index");
  if (n < 0 || i0 < 0 || i0 + n > idx->ntotal)
    return fail(VS_E_INVALID, "vs_reconstruct_n: key out of range");  // faiss: FAISS_THROW_IF_NOT
  if (n == 0) return VS_OK;
  if (!out) return fail(VS_E_INVALID, "vs_reconstruct_n: null output");
  hipStream_t st = (hipStream_t)stream;
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  const hipMemcpyKind kind =
      (flags & VS_OUT_DEVICE) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (idx->esize == 4) {
    VS_HIP(hipMemcpy2DAsync(out, (size_t)idx->d * sizeof(float), idx->row(i0), idx->rowbytes(),
                            (size_t)idx->d * sizeof(float), (size_t)n, kind, st),
           "vs_reconstruct_n: copy");
  } else {
    // widen bf16 rows in bounded chunks, then copy out
    const int64_t chunk = std::max<int64_t>(1, (int64_t)(64ull << 20) / (idx->d * 4));
    Scratch scr(st);
    float* tmp = nullptr;
    VS_HIP(scr.alloc((void**)&tmp, (size_t)std::min(chunk, n) * idx->d * sizeof(float)),
           "vs_reconstruct_n: scratch");
    for (int64_t r0 = 0; r0 < n; r0 += chunk) {
      const int64_t m = std::min(chunk, n - r0);
      VS_HIP(launch_bf16_to_f32((const uint16_t*)idx->row(i0 + r0), idx->ld, tmp, idx->d, m,
                                idx->d, st),
             "vs_reconstruct_n: widen");
      VS_HIP(hipMemcpyAsync(out + r0 * idx->d, tmp, (size_t)m * idx->d * sizeof(float), kind, st),
             "vs_reconstruct_n: copy");
    }
    VS_HIP(hipStreamSynchronize(st), "vs_reconstruct_n: synchronise");
  }
  if (!(flags & VS_OUT_DEVICE)) VS_HIP(hipStreamSynchronize(st), "vs_reconstruct_n: synchronise");
  return VS_OK;
}

int vs_remove_ids(vs_index* idx, const int64_t* ids, int64_t n, int64_t* nremoved) {
  if (!idx) return fail(VS_E_INVALID, "vs_remove_ids: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_remove_ids: n < 0");
  if (nremoved) *nremoved = 0;
  if (n == 0) return VS_OK;
  if (!ids) return fail(VS_E_INVALID, "vs_remove_ids: null ids");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  // IDSelectorBatch semantics: membership test; duplicates and out-of-range ids
  // are ignored.  Labels here are global (id_base applied), as faiss sees them.
  std::vector<int64_t> rm;
  rm.reserve((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = ids[i] - idx->id_base;
    if (r >= 0 && r < idx->ntotal) rm.push_back(r);
  }
  std::sort(rm.begin(), rm.end());
  rm.erase(std::unique(rm.begin(), rm.end()), rm.end());
  const int64_t nrem = (int64_t)rm.size();
  if (nrem == 0) return VS_OK;
  DeviceGuard g(idx->device);
  // Searches already queued on other streams read the rows we are about to move.
  VS_HIP(hipDeviceSynchronize(), "vs_remove_ids: drain");
  hipStream_t st = nullptr;
  Scratch scr(st);
  int64_t* drm = nullptr;
  VS_HIP(scr.alloc((void**)&drm, (size_t)nrem * sizeof(int64_t)), "vs_remove_ids: scratch");
  VS_HIP(hipMemcpyAsync(drm, rm.data(), (size_t)nrem * sizeof(int64_t), hipMemcpyHostToDevice, st),
         "vs_remove_ids: upload");
  // Chunked stable compaction from the first removed row on: each chunk's kept
  // rows are packed into scratch, then copied down to their final position.
  // Destinations never exceed the chunk's own source range, and earlier chunks
  // are already consumed, so the in-place move is safe with O(chunk) scratch.
  const int64_t chunk = std::max<int64_t>(1024, (int64_t)(256ull << 20) / idx->rowbytes());
  char* tmp = nullptr;
  float* tmpn = nullptr;
  VS_HIP(scr.alloc((void**)&tmp, (size_t)chunk * idx->rowbytes()), "vs_remove_ids: scratch");
  VS_HIP(scr.alloc((void**)&tmpn, (size_t)chunk * sizeof(float)), "vs_remove_ids: scratch");
  const int64_t first = rm[0];
  for (int64_t s0 = first; s0 < idx->ntotal; s0 += chunk) {
    const int64_t cn = std::min(chunk, idx->ntotal - s0);
    const int64_t before = std::lower_bound(rm.begin(), rm.end(), s0) - rm.begin();
    const int64_t in_chunk = std::lower_bound(rm.begin(), rm.end(), s0 + cn) - rm.begin() - before;
    const int64_t kept = cn - in_chunk;
    const int64_t dst = s0 - before;
    VS_HIP(launch_gather_kept(idx->codes, idx->norms, idx->rowbytes(), s0, cn, drm, nrem, tmp, tmpn,
                              st),
           "vs_remove_ids: gather");
    if (kept > 0) {
      VS_HIP(hipMemcpyAsync(idx->row(dst), tmp, (size_t)kept * idx->rowbytes(),
                            hipMemcpyDeviceToDevice, st),
             "vs_remove_ids: move rows");
      VS_HIP(hipMemcpyAsync(idx->norms + dst, tmpn, (size_t)kept * sizeof(float),
                            hipMemcpyDeviceToDevice, st),
             "vs_remove_ids: move norms");
    }
  }
  const int64_t nt = idx->ntotal - nrem;
  idx->blocked_rows = std::min(idx->blocked_rows, first);  // rows from `first` on moved
  idx->planes_rows = std::min(idx->planes_rows, first);
  VS_HIP(hipMemsetAsync(idx->row(nt), 0, (size_t)nrem * idx->rowbytes(), st),
         "vs_remove_ids: zero tail");
  VS_HIP(hipMemsetAsync(idx->norms + nt, 0, (size_t)nrem * sizeof(float), st),
         "vs_remove_ids: zero tail");
  VS_HIP(hipStreamSynchronize(st), "vs_remove_ids: synchronise");
  idx->ntotal = nt;
  if (nremoved) *nremoved = nrem;
  return VS_OK;
}

int vs_selfjoin(vs_index* idx, int64_t q0, int64_t nq, int64_t k, int exclude_self,
                float min_sim, float* D, int64_t* I, int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_selfjoin: null index");
  if (k <= 0) return fail(VS_E_INVALID, "vs_selfjoin: k must be > 0");
  if (k > VS_MAX_K) return fail(VS_E_UNSUPPORTED, "vs_selfjoin: k > VS_MAX_K (64) not supported yet");
  if (q0 < 0 || nq < 0 || q0 + nq > idx->ntotal)
    return fail(VS_E_INVALID, "vs_selfjoin: query rows out of range");
  if (nq == 0) return VS_OK;
  if (!D || !I) return fail(VS_E_INVALID, "vs_selfjoin: null buffer");
  hipStream_t st = (hipStream_t)stream;
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  const bool out_dev = (flags & VS_OUT_DEVICE) != 0;
  Scratch scr(st);
  float* Dd = D;
  int64_t* Id = I;
  if (!out_dev) {
    VS_HIP(scr.alloc((void**)&Dd, (size_t)nq * k * sizeof(float)), "vs_selfjoin: scratch");
    VS_HIP(scr.alloc((void**)&Id, (size_t)nq * k * sizeof(int64_t)), "vs_selfjoin: scratch");
  }
  float* rinv = nullptr;
  VS_HIP(scr.alloc((void**)&rinv, (size_t)idx->capacity * sizeof(float)), "vs_selfjoin: scratch");
  VS_HIP(launch_rsqrt(idx->norms, idx->capacity, rinv, st), "vs_selfjoin: rsqrt");
  // Query tiles read stored rows directly (capacity keeps kBQ rows of slack).
  const int64_t chunk = 65536;
  for (int64_t c0 = 0; c0 < nq; c0 += chunk) {
    const int64_t nc = std::min(chunk, nq - c0);
    const int64_t nq_pad = round_up(nc, kBQ);
    const int64_t qrow = q0 + c0;
    const bool b16 = idx->esize == 2;
    int rc = run_topk(idx, MODE_COS, b16 ? nullptr : (const float*)idx->row(qrow),
                      b16 ? (const void*)idx->row(qrow) : nullptr, rinv + qrow, (int)nc,
                      (int)nq_pad, (int)k, exclude_self ? qrow : -1, min_sim, Dd + c0 * k,
                      Id + c0 * k, st, rinv);
    if (rc) return rc;
  }
  if (!out_dev) {
    VS_HIP(hipMemcpyAsync(D, Dd, (size_t)nq * k * sizeof(float), hipMemcpyDeviceToHost, st),
           "vs_selfjoin: copy D");
    VS_HIP(hipMemcpyAsync(I, Id, (size_t)nq * k * sizeof(int64_t), hipMemcpyDeviceToHost, st),
           "vs_selfjoin: copy I");
    VS_HIP(hipStreamSynchronize(st), "vs_selfjoin: synchronise");
  }
  return VS_OK;
}

int vs_merge_topk(const float* D_parts, const int64_t* I_parts, int64_t nparts, int64_t nq,
                  int64_t k_in, int64_t k, int metric, float* D, int64_t* I, void* stream) {
  if (nparts < 1 || nq < 0 || k_in < 1 || k < 1)
    return fail(VS_E_INVALID, "vs_merge_topk: bad sizes");
  if (k > VS_MAX_K) return fail(VS_E_UNSUPPORTED, "vs_merge_topk: k > VS_MAX_K");
  if (metric != VS_METRIC_L2 && metric != VS_METRIC_INNER_PRODUCT)
    return fail(VS_E_INVALID, "vs_merge_topk: bad metric");
  if (nq == 0) return VS_OK;
  if (!D_parts || !I_parts || !D || !I) return fail(VS_E_INVALID, "vs_merge_topk: null buffer");
  VS_HIP(launch_merge_parts(metric == VS_METRIC_L2 ? MODE_L2 : MODE_IP, D_parts, I_parts,
                            (int)nparts, (int)nq, (int)k_in, (int)k, D, I, (hipStream_t)stream),
         "vs_merge_topk: launch");
  return VS_OK;
}

int vs_fill_synthetic(float* out, int64_t rows, int64_t d, uint64_t seed, int64_t row0,
                      void* stream) {
  if (rows < 0 || d <= 0 || row0 < 0) return fail(VS_E_INVALID, "vs_fill_synthetic: bad sizes");
  if (rows == 0) return VS_OK;
  if (!out) return fail(VS_E_INVALID, "vs_fill_synthetic: null output");
  VS_HIP(launch_fill_synthetic(out, 4, rows, d, d, seed, row0, (hipStream_t)stream),
         "vs_fill_synthetic: launch");
  return VS_OK;
}

int vs_filter_stats(int64_t* queries, int64_t* fallbacks, int reset) {
  if (!queries || !fallbacks) return fail(VS_E_INVALID, "vs_filter_stats: null output");
  std::lock_guard<std::mutex> g(g_timer_mu);
  *queries = g_filter_queries;
  *fallbacks = g_filter_fallbacks;
  if (reset) g_filter_queries = g_filter_fallbacks = g_filter_wide = 0;
  return VS_OK;
}

int vs_filter_wide_stats(int64_t* wide) {
  if (!wide) return fail(VS_E_INVALID, "vs_filter_wide_stats: null output");
  std::lock_guard<std::mutex> g(g_timer_mu);
  *wide = g_filter_wide;
  return VS_OK;
}

int vs_timer_enable(int on) {
  std::lock_guard<std::mutex> g(g_timer_mu);
  g_timer_on = on != 0;
  return VS_OK;
}

int vs_timer_reset(void) {
  std::lock_guard<std::mutex> g(g_timer_mu);
  for (auto& p : g_timer_events) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  g_timer_events.clear();
  return VS_OK;
}

const char* vs_timer_kernel(void) {
  std::lock_guard<std::mutex> g(g_timer_mu);
  return g_timer_kernel;
}

int vs_timer_read(double* total_ms, int64_t* launches) {
  if (!total_ms || !launches) return fail(VS_E_INVALID, "vs_timer_read: null output");
  std::lock_guard<std::mutex> g(g_timer_mu);
  double tot = 0.0;
  int64_t n = 0;
  for (auto& p : g_timer_events) {
    VS_HIP(hipEventSynchronize(p.b), "vs_timer_read: synchronise");
    float ms = 0.0f;
    VS_HIP(hipEventElapsedTime(&ms, p.a, p.b), "vs_timer_read: elapsed");
    tot += ms;
    n += p.dispatches;
  }
  *total_ms = tot;
  *launches = n;
  return VS_OK;
}

}  // extern "C"
