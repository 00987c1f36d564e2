// vs_api.hip — the C-ABI of libvsearch.so (declared in include/vsearch.h).
//
// A vs_index is one device's exact flat index: library-owned row storage in HBM
// (fp32 or bf16 elements, stride `ld` elements = a multiple of 128 B, zero
// padding), the squared norms of every row, and ntotal.  It mirrors faiss::IndexFlat (faiss-cpu 1.11.0, not vendored; see
// /root/reference/poetry.lock:866-867): add copies the caller's rows, search
// writes caller-allocated D/I, remove_ids compacts stably.
//
// Concurrency follows faiss's contract (concurrent searches allowed, add/remove
// exclusive): a shared_mutex guards the storage; per-call scratch comes from a
// chunk cache whose chunks carry the event of their last use, so a search on
// another stream waits (on the device) before it reuses one.
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

// bf16-first searches between int8 probes: the first gap, doubling to the last.
constexpr int kI8FirstBackoff = 8;
constexpr int kI8MaxBackoff = 64;

struct vs_index {
  int d = 0;
  int metric = VS_METRIC_L2;
  int dtype = VS_DTYPE_F32;
  int device = 0;
  int esize = 4;         // bytes per stored element (4 fp32, 2 bf16)
  int64_t ld = 0;        // row stride in elements, a multiple of 64 (zero padding)
  int64_t ntotal = 0;
  int64_t capacity = 0;  // rows allocated (multiple of kRowPad, >= ntotal + 256)
  int64_t id_base = 0;
  char* codes = nullptr;   // [capacity][ld] elements
  int64_t rowbytes() const { return ld * esize; }
  char* row(int64_t r) const { return codes + r * rowbytes(); }
  float* norms = nullptr;  // [capacity] squared L2 norms
  // fp32 indexes: the filter planes the filter passes multiply ([capacity][ld]
  // each, kept in step with the rows by add / remove_ids / growth) and
  // |x - plane(x)|^2 per row for the bound: [FILTER_I8] int8 codes + a per-row
  // scale (inner-product indexes), [FILTER_BF16] bf16 (round-to-nearest-even)
  // copies.  bf16 indexes use the exact bf16 engine, no plane.
  bool plane_on[2] = {false, false};
  char* fplane[2] = {nullptr, nullptr};
  float* rn2[2] = {nullptr, nullptr};
  float* fscale = nullptr;  // int8 plane: s = max|x| / 127 per row
  // per plane: max |x|^2, max |x - plane(x)|^2, max of their ratio over the
  // rows (the bound's index maxima; grown by add, recomputed by remove_ids)
  unsigned* bstats[2] = {nullptr, nullptr};
  // L2 indexes: both planes hold augmented rows x' = [x, e_1 .. e_m] whose
  // inner product with q' = [q, C .. C] ranks rows as the L2 key does
  // (launch_quantize_i8_l2aug, launch_bf16_plane_l2aug); the parameters are
  // set by the first add (aug_m = 0 before), anorm / anorm_b = |x'|^2 per row
  // (the planes' bound maxima use them)
  int aug_m = 0;
  L2Aug aug;
  float* anorm = nullptr;
  float* anorm_b = nullptr;
  // Tombstones (indexes without filter planes, e.g. bf16 storage): removed
  // rows stay in place, NaN-filled (no kernel admits them), until a pack; faiss
  // labels are positions among the live rows (searches map their rows through
  // the sorted dead list, launch_label_map).  ntotal counts the rows in place.
  std::string notice;  // the last plane loss (vs_notice), empty if none
  std::vector<int64_t> dead;
  int64_t* ddead = nullptr;  // device copy of `dead`
  int64_t ddead_cap = 0;
  int64_t live() const { return ntotal - (int64_t)dead.size(); }
  // removals fill rows with NaN in place (labels mapped at search time) instead
  // of compacting at once: bf16 indexes (C5: 154 GB of rows cannot move at every
  // removal; an int8 plane of theirs has its factors set to NaN with them) and
  // indexes without planes
  bool tombstones() const { return esize == 2 || (!plane_on[0] && !plane_on[1]); }
  bool l2aug() const { return metric == VS_METRIC_L2 && esize == 4; }
  int64_t planebytes(int p) const {
    if (!l2aug()) return ld * filter_bytes(p);
    return (p == FILTER_I8 ? ld + aug_m : ld + kAugBf16) * filter_bytes(p);
  }
  // Adaptive plane order: the int8 stage pays off while it settles most
  // queries; on data where it hands most of them to bf16 (clustered
  // embeddings) the searches go to bf16 directly, re-probing int8 with an
  // exponential backoff.  Device counters [i8 queries, handed to bf16], read
  // through a pinned mirror when the copy's event has completed (no host wait).
  struct Adaptive {
    std::mutex mu;
    unsigned long long* dcount = nullptr;
    unsigned long long* hmirror = nullptr;
    hipEvent_t ev = nullptr;
    bool pending = false;
    unsigned long long seen_q = 0, seen_h = 0;
    double ema = 0.0;
    bool have = false;
    int skip_left = 0, backoff = kI8FirstBackoff;
  } ad;
  int engine = VS_ENGINE_AUTO;
  std::shared_mutex mu;
  // Completion marks of the calls that read this index's storage on the
  // device: one event per stream a search / self-join / device reconstruct ran
  // on, recorded after its last launch.  Writers that move or free the storage
  // (growth, remove_ids, reset, destroy) wait for these marks only — not for
  // the whole device, where other indexes' searches may be running (faiss's
  // contract: a writer excludes the readers of its own index).
  std::mutex rd_mu;
  std::vector<std::pair<hipStream_t, hipEvent_t>> readers;
  hipStream_t wst = nullptr;  // the index's own (non-blocking) writer stream
};

namespace {

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

// Records a reader mark of `idx` on `st` when it leaves scope (after the
// caller's last launch on st; also on an error return).
struct ReaderMark {
  vs_index* idx;
  hipStream_t st;
  ReaderMark(vs_index* i, hipStream_t s) : idx(i), st(s) {}
  ~ReaderMark() {
    std::lock_guard<std::mutex> g(idx->rd_mu);
    for (auto& r : idx->readers)
      if (r.first == st) {
        (void)hipEventRecord(r.second, st);
        return;
      }
    // a new stream: first drop the marks that have completed (a caller with a
    // stream per request would otherwise grow the list, and every writer's
    // wait_readers, without bound)
    for (size_t i = 0; i < idx->readers.size();) {
      if (hipEventQuery(idx->readers[i].second) == hipSuccess) {
        (void)hipEventDestroy(idx->readers[i].second);
        idx->readers[i] = idx->readers.back();
        idx->readers.pop_back();
      } else {
        ++i;
      }
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(st);  // no mark possible: finish the work instead
      return;
    }
    (void)hipEventRecord(ev, st);
    idx->readers.emplace_back(st, ev);
  }
};

// Waits (host) until every reader mark of `idx` has completed.  Called with
// the index's writer lock held, so no new reader can start meanwhile.
hipError_t wait_readers(vs_index* idx) {
  std::lock_guard<std::mutex> g(idx->rd_mu);
  for (auto& r : idx->readers) {
    hipError_t e = hipEventSynchronize(r.second);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The index's writer stream (created on first use): non-blocking, so it never
// serialises with the legacy null stream's users, and of the greatest
// priority, which gives it a hardware queue of its own — streams of one
// priority share the process's few hardware queues (GPU_MAX_HW_QUEUES), and a
// shared queue would run the writer behind another stream's search queue.
hipError_t writer_stream(vs_index* idx, hipStream_t* out) {
  if (!idx->wst) {
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return e;
    e = hipStreamCreateWithPriority(&idx->wst, hipStreamNonBlocking, greatest);
    if (e != hipSuccess) return e;
  }
  *out = idx->wst;
  return hipSuccess;
}

// Stream-ordered scratch allocation, released on scope exit (on the same stream;
// the device's default pool keeps the memory cached, vs_create).
// Scratch chunks (vs_internal.h): power-of-two sizes from 64 MB, kept after
// use with the event of their last use; a taker's stream waits on that event
// (a device-side wait).  The stream-ordered allocator cost ~76 us of host time
// per hipFreeAsync at C2 (the search loop was host-bound: 2.6 ms of host per
// 2.45 ms of kernels) and ~12 ms per call on C4's large lists (rocprofv3
// --hip-trace, profiles/r02zl, r02zm).
}  // namespace (the chunk cache is shared with vs_support.hip)

namespace {
std::mutex g_chunk_mu;
std::vector<ScratchChunk> g_chunk_idle;
size_t g_chunk_idle_bytes = 0;
constexpr size_t kChunkMin = size_t(64) << 20;
constexpr size_t kChunkIdleCap = size_t(16) << 30;  // per process
}  // namespace

namespace vs {
void scratch_trim() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::vector<ScratchChunk> drop;
  {
    std::lock_guard<std::mutex> g(g_chunk_mu);
    for (size_t i = 0; i < g_chunk_idle.size();) {
      if (g_chunk_idle[i].dev == dev) {
        drop.push_back(g_chunk_idle[i]);
        g_chunk_idle_bytes -= g_chunk_idle[i].size;
        g_chunk_idle[i] = g_chunk_idle.back();
        g_chunk_idle.pop_back();
      } else {
        ++i;
      }
    }
  }
  if (drop.empty()) return;
  for (auto& c : drop) (void)hipEventSynchronize(c.ev);  // each chunk's last use
  for (auto& c : drop) {
    (void)hipFree(c.p);
    (void)hipEventDestroy(c.ev);
  }
}

hipError_t scratch_chunk_get(size_t bytes, hipStream_t st, ScratchChunk* out) {
  size_t sz = kChunkMin;
  while (sz < bytes) sz <<= 1;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  // An idle chunk last used on this stream needs no wait (stream order), one
  // whose last use has completed needs none either; a chunk still in use on
  // another stream would tie this call to that stream's queue (another
  // index's long searches, say), so a new chunk is allocated instead while
  // memory allows, and only then is the busy one taken with a device-side wait.
  int busy = -1;
  {
    std::lock_guard<std::mutex> g(g_chunk_mu);
    int pick = -1;
    for (size_t i = 0; i < g_chunk_idle.size(); ++i) {
      const ScratchChunk& c = g_chunk_idle[i];
      // the power-of-two chunk of this request, or an exact-size one (the OOM
      // fallback below) that holds it
      if (c.dev != dev || c.size < bytes || c.size > sz) continue;
      if (c.st == st || hipEventQuery(c.ev) == hipSuccess) {
        pick = (int)i;
        break;
      }
      if (busy < 0) busy = (int)i;
    }
    (void)hipGetLastError();  // hipEventQuery's hipErrorNotReady
    if (pick >= 0) {
      *out = g_chunk_idle[pick];
      g_chunk_idle[pick] = g_chunk_idle.back();
      g_chunk_idle.pop_back();
      g_chunk_idle_bytes -= out->size;
      return out->st == st ? hipSuccess : hipStreamWaitEvent(st, out->ev, 0);
    }
  }
  ScratchChunk c;
  c.size = sz;
  c.dev = dev;
  e = hipMalloc(&c.p, sz);
  if (e != hipSuccess && busy >= 0) {  // short of memory: wait for the busy chunk
    (void)hipGetLastError();
    std::lock_guard<std::mutex> g(g_chunk_mu);
    for (size_t i = 0; i < g_chunk_idle.size(); ++i) {
      if (g_chunk_idle[i].dev == dev && g_chunk_idle[i].size >= bytes &&
          g_chunk_idle[i].size <= sz) {
        *out = g_chunk_idle[i];
        g_chunk_idle[i] = g_chunk_idle.back();
        g_chunk_idle.pop_back();
        g_chunk_idle_bytes -= out->size;
        return hipStreamWaitEvent(st, out->ev, 0);
      }
    }
  }
  if (e != hipSuccess) {  // idle chunks of other sizes may hold the memory
    (void)hipGetLastError();
    scratch_trim();
    e = hipMalloc(&c.p, sz);
  }
  if (e != hipSuccess) {  // the power-of-two rounding may be what does not fit
    (void)hipGetLastError();
    const size_t exact = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    if (exact >= sz) return e;
    c.size = exact;
    e = hipMalloc(&c.p, exact);
    if (e != hipSuccess) return e;
  }
  e = hipEventCreateWithFlags(&c.ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    (void)hipFree(c.p);
    return e;
  }
  *out = c;
  return hipSuccess;
}

void scratch_chunk_put(const ScratchChunk& c0, hipStream_t st) {
  if (!c0.p) return;
  ScratchChunk c = c0;
  c.st = st;
  (void)hipEventRecord(c.ev, st);
  {
    std::lock_guard<std::mutex> g(g_chunk_mu);
    if (g_chunk_idle_bytes + c.size <= kChunkIdleCap) {
      g_chunk_idle.push_back(c);
      g_chunk_idle_bytes += c.size;
      return;
    }
  }
  (void)hipEventSynchronize(c.ev);
  (void)hipFree(c.p);
  (void)hipEventDestroy(c.ev);
}
}  // namespace vs

namespace {

// Per-call scratch: bump allocation from cached chunks, returned at scope end.
struct Scratch {
  static constexpr size_t kAlign = 256;
  hipStream_t st;
  std::vector<ScratchChunk> chunks;
  char* cur = nullptr;
  size_t left = 0;
  explicit Scratch(hipStream_t s) : st(s) {}
  hipError_t alloc(void** p, size_t bytes) {
    *p = nullptr;
    if (bytes == 0) return hipSuccess;
    bytes = (bytes + kAlign - 1) & ~(kAlign - 1);
    if (bytes > left) {
      ScratchChunk c;
      hipError_t e = scratch_chunk_get(bytes, st, &c);
      if (e != hipSuccess) return e;
      chunks.push_back(c);
      cur = (char*)c.p;
      left = c.size;
    }
    *p = cur;
    cur += bytes;
    left -= bytes;
    return hipSuccess;
  }
  ~Scratch() {
    for (auto& c : chunks) scratch_chunk_put(c, st);
  }
};

// Kernel timer (measurement hook for bench.py; see vs_timer_* in vsearch.h).
std::mutex g_timer_mu;
bool g_timer_on = false;
struct TimedSpan {
  hipEvent_t a, b;
  int dispatches;
  const char* name;
  bool aux;      // an extra span over other spans' kernels: not in the unnamed total
  double share;  // the span's share of its pass's database tiles (filter passes)
};
std::vector<TimedSpan> g_timer_events;
const char* g_timer_kernel = "";

// Filter-and-verify statistics, counted on the device (no host sync in a
// search): [0] queries, [1] flagged by the first check (given to the wide
// check), [2] flagged by both (redone by the exact engine), [3] handed to a
// second filter stage, [4] wide-set entries, [5] of them rescored (the rest
// reuse the first check's keys), [6] rows stored by dump launches (one
// (row, raw sum) slot each), [7] lane lists out of dump slots.  One buffer per device.
constexpr int kStatSlots = 9;  // [8]: queries ranked by the exact-key stream
std::mutex g_stats_mu;
std::vector<unsigned long long*> g_dev_stats;

unsigned long long* device_stats(int dev) {
  std::lock_guard<std::mutex> g(g_stats_mu);
  if ((int)g_dev_stats.size() <= dev) g_dev_stats.resize(dev + 1, nullptr);
  if (!g_dev_stats[dev]) {
    unsigned long long* p = nullptr;
    if (hipMalloc(&p, kStatSlots * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    if (hipMemset(p, 0, kStatSlots * sizeof(unsigned long long)) != hipSuccess) return nullptr;
    g_dev_stats[dev] = p;
  }
  return g_dev_stats[dev];
}

// The wide verification of flagged queries (VS_X1_WIDE=0 turns it off, for A/B).
bool wide_enabled() {
  static const bool on = [] {
    const char* e = getenv("VS_X1_WIDE");
    return !(e && e[0] == '0');
  }();
  return on;
}

struct KernelTimer {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  const char* name = nullptr;
  int dispatches = 1;  // kernel launches between the two events
  bool aux = false;
  double share = 1.0;  // of a filter pass's tiles (X1SpanTimer)
  // name == nullptr: untimed (the filter engine's exact redo, which is not the
  // kernel the roofline is quoted on)
  // names_kernel: this span names the search's dominant kernel (vs_timer_kernel);
  // false for an extra span over several kernels (the whole filter pass)
  KernelTimer(hipStream_t s, const char* nm, bool names_kernel = true) : st(s), name(nm) {
    if (!name) return;
    std::lock_guard<std::mutex> g(g_timer_mu);
    if (names_kernel) g_timer_kernel = name;
    aux = !names_kernel;
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
    g_timer_events.push_back({a, b, dispatches, name, aux, share});
    a = b = nullptr;
  }
};

// The filter pass's per-launch spans: dump launches (and every launch of a
// pass without dumps) under the pass's timer name, the list launch of a pass
// with dumps under "<name>_list" (bench.py: the roofline is the dominant
// kernel's own time; the cut and replay kernels between launches are in no
// span).
struct X1SpanTimer : X1Timing {
  const char* name;
  const char* list_name;
  KernelTimer* cur = nullptr;
  X1SpanTimer(const char* n, const char* ln) : name(n), list_name(ln) {}
  void begin(hipStream_t st, bool dominant, double share) override {
    cur = new KernelTimer(st, dominant ? name : list_name);
    cur->share = share;
  }
  void end(hipStream_t) override {
    if (!cur) return;
    cur->stop();
    delete cur;
    cur = nullptr;
  }
  ~X1SpanTimer() override { end(nullptr); }
};

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

int kp_for(int64_t k) {
  return k <= 8      ? 8
         : k <= 16   ? 16
         : k <= 32   ? 32
         : k <= 64   ? 64
         : k <= 128  ? 128
         : k <= 256  ? 256
         : k <= 512  ? 512
                     : 1024;
}

int engine_from_env() {
  const char* e = getenv("VS_ENGINE");
  if (!e) return VS_ENGINE_AUTO;
  if (strcmp(e, "fp32") == 0) return VS_ENGINE_FP32_MFMA;
  if (strcmp(e, "bf16v") == 0) return VS_ENGINE_BF16_VERIFY;
  if (strcmp(e, "i8v") == 0) return VS_ENGINE_I8_VERIFY;
  return VS_ENGINE_AUTO;
}

// Filter planes of a new fp32 index: int8 + bf16 (the staged engine; an L2
// index's int8 plane holds the augmented rows, vs_index::aug_m).  Env
// VS_FILTER=bf16 | i8 keeps only that plane (A/B).
void planes_for(vs_index* idx) {
  const char* e = getenv("VS_FILTER");
  if (e && strcmp(e, "none") == 0) {  // no planes: the exact fp32 engine alone
    idx->plane_on[FILTER_BF16] = idx->plane_on[FILTER_I8] = false;
    return;
  }
  const bool f32 = idx->esize == 4;
  // bf16 indexes: an int8 plane for inner product (C5: the small-batch filter
  // pass streams 1 B per element instead of the rows' 2; the verification
  // rescores the stored bf16 values)
  const bool i8able = f32 ? (idx->metric == VS_METRIC_INNER_PRODUCT || idx->metric == VS_METRIC_L2)
                          : idx->metric == VS_METRIC_INNER_PRODUCT;
  idx->plane_on[FILTER_BF16] = f32 && !(i8able && e && strcmp(e, "i8") == 0);
  idx->plane_on[FILTER_I8] = i8able && !(e && strcmp(e, "bf16") == 0);
}

// An L2 index without rows forgets its augmentation (vs_reset, or removals
// down to ntotal = 0): the first add after it chooses m, C and nref again.
void reset_l2aug(vs_index* idx) {
  idx->aug_m = 0;
  idx->aug = L2Aug{};
}

// The augmentation of an L2 index's int8 plane, fixed by its first add (rows
// [0, n) in place, their norms too): m extra columns and C (l2aug_params),
// then the plane reallocated at ld + m bytes per row (it holds no row yet).
int choose_l2aug(vs_index* idx, int64_t n, hipStream_t st) {
  L2Aug g;
  VS_HIP(l2aug_params((const float*)idx->codes, idx->ld, 0, n, idx->norms, &g, st),
         "vs: L2 plane parameters");
  VS_HIP(hipStreamSynchronize(st), "vs: L2 plane");
  if (!idx->plane_on[FILTER_I8]) {  // the bf16 plane's width does not depend on them
    idx->aug_m = g.m;
    idx->aug = g;
    return VS_OK;
  }
  VS_HIP(wait_readers(idx), "vs: L2 plane");
  if (idx->fplane[FILTER_I8]) (void)hipFree(idx->fplane[FILTER_I8]);
  idx->fplane[FILTER_I8] = nullptr;
  idx->aug_m = g.m;
  idx->aug = g;
  hipError_t e = hipMalloc(&idx->fplane[FILTER_I8], (size_t)idx->capacity * idx->planebytes(FILTER_I8));
  if (e != hipSuccess) {  // no room for the wider plane: the index goes on without it
    (void)hipGetLastError();
    idx->fplane[FILTER_I8] = nullptr;
    idx->plane_on[FILTER_I8] = false;
    return VS_OK;
  }
  VS_HIP(launch_plane_zero_rows(idx->fplane[FILTER_I8], idx->planebytes(FILTER_I8), 0,
                                idx->capacity, st),
         "vs: L2 plane");
  return VS_OK;
}

// The norms a plane's bound maxima take: |x'|^2 for an L2 index's augmented
// int8 plane, the stored |x|^2 otherwise.
const float* plane_norms(const vs_index* idx, int p) {
  if (!idx->l2aug()) return idx->norms;
  return p == FILTER_I8 ? idx->anorm : idx->anorm_b;
}

// The filter plane and residual norms of fp32 rows [r0, r0+n) (after the rows
// and their norms are in place).
int derive_plane(vs_index* idx, int64_t r0, int64_t n, hipStream_t st, bool appended = false) {
  if (n <= 0 || (idx->esize != 4 && !idx->plane_on[FILTER_I8])) return VS_OK;
  for (int p = 0; p < 2; ++p) {
    if (!idx->plane_on[p] || idx->bstats[p]) continue;
    VS_HIP(hipMalloc(&idx->bstats[p], 4 * sizeof(unsigned)), "vs: bound maxima");
    VS_HIP(hipMemsetAsync(idx->bstats[p], 0, 4 * sizeof(unsigned), st), "vs: bound maxima");
  }
  // An add that at least doubles an L2 index re-derives its augmentation over
  // every row (a few first rows would otherwise fix m, C and nref for good, and
  // rows of other norms get coarse codes and a wide bound); amortised O(1) per
  // row, like the storage's own growth.
  if (appended && idx->l2aug() && idx->aug_m > 0 && r0 > 0 && n >= r0) {
    reset_l2aug(idx);
    for (int p = 0; p < 2; ++p)
      if (idx->bstats[p])
        VS_HIP(hipMemsetAsync(idx->bstats[p], 0, 4 * sizeof(unsigned), st), "vs: bound maxima");
  }
  if (idx->l2aug() && idx->aug_m == 0 && (idx->plane_on[FILTER_I8] || idx->plane_on[FILTER_BF16])) {
    // the first rows fix the augmentation (and the int8 plane's width)
    const int64_t n0 = r0 + n;
    int rc = choose_l2aug(idx, n0, st);
    if (rc) return rc;
    r0 = 0;
    n = n0;
  }
  if (idx->plane_on[FILTER_I8] && idx->l2aug()) {
    if (idx->plane_on[FILTER_I8])
      VS_HIP(launch_quantize_i8_l2aug((const float*)idx->codes, idx->ld, r0, n, idx->aug,
                                      idx->norms, (int8_t*)idx->fplane[FILTER_I8], idx->fscale,
                                      idx->rn2[FILTER_I8], idx->anorm, st),
             "vs: int8 L2 filter plane");
  } else if (idx->plane_on[FILTER_I8]) {
    VS_HIP(launch_quantize_i8(idx->codes, idx->ld, r0, n, (int8_t*)idx->fplane[FILTER_I8],
                              idx->fscale, idx->rn2[FILTER_I8], st, idx->esize),
           "vs: int8 filter plane");
  }
  if (idx->plane_on[FILTER_BF16] && idx->l2aug()) {
    VS_HIP(launch_bf16_plane_l2aug((const float*)idx->codes, idx->ld, r0, n, idx->aug, idx->norms,
                                   (uint16_t*)idx->fplane[FILTER_BF16], idx->rn2[FILTER_BF16],
                                   idx->anorm_b, st),
           "vs: bf16 L2 filter plane");
  } else if (idx->plane_on[FILTER_BF16]) {
    VS_HIP(launch_bf16_plane((const float*)idx->codes, idx->ld, r0, n,
                             (uint16_t*)idx->fplane[FILTER_BF16], st),
           "vs: bf16 filter plane");
    VS_HIP(launch_resid_norms((const float*)idx->codes, idx->ld, r0, n, idx->rn2[FILTER_BF16], st),
           "vs: residual norms");
  }
  // the new rows' maxima fold into the index's (they only grow on add)
  for (int p = 0; p < 2; ++p)
    if (idx->plane_on[p])
      VS_HIP(launch_bound_stats(plane_norms(idx, p) + r0, idx->rn2[p] + r0, n, idx->bstats[p], st,
                                true),
             "vs: bound maxima");
  return VS_OK;
}

void free_storage(vs_index* idx);

// Grows storage to hold `rows` rows (plus the tile slack), preserving content.
int ensure_capacity(vs_index* idx, int64_t rows, hipStream_t st) {
  const int64_t need = round_up(rows + 256, kRowPad);  // 256-row query tiles of self-joins
  if (need <= idx->capacity) return VS_OK;
  int64_t cap = std::max(need, round_up(idx->capacity + idx->capacity / 2, kRowPad));
  char* codes = nullptr;
  float* norms = nullptr;
  char* fplane[2] = {nullptr, nullptr};
  float* rn2[2] = {nullptr, nullptr};
  float* fscale = nullptr;
  float* anorm = nullptr;
  float* anorm_b = nullptr;
  // the planes the new storage keeps: committed to the index only once the
  // allocation succeeded (a failed growth leaves the index as it was)
  bool on[2] = {idx->plane_on[0], idx->plane_on[1]};
  auto release = [&]() {
    if (codes) (void)hipFree(codes);
    if (norms) (void)hipFree(norms);
    for (int p = 0; p < 2; ++p) {
      if (fplane[p]) (void)hipFree(fplane[p]);
      if (rn2[p]) (void)hipFree(rn2[p]);
      fplane[p] = nullptr;
      rn2[p] = nullptr;
    }
    if (fscale) (void)hipFree(fscale);
    if (anorm) (void)hipFree(anorm);
    if (anorm_b) (void)hipFree(anorm_b);
    codes = nullptr;
    norms = nullptr;
    fscale = nullptr;
    anorm = nullptr;
    anorm_b = nullptr;
  };
  // test hook (tests/test_gpu_planes.py): VS_TEST_PLANE_OOM=1 fails the bf16
  // plane's allocation as a full HBM would, 2 every plane's
  static const int plane_oom = [] {
    const char* v = getenv("VS_TEST_PLANE_OOM");
    return v ? atoi(v) : 0;
  }();
  auto allocate = [&](int64_t c) -> hipError_t {
    hipError_t e = hipMalloc(&codes, (size_t)c * idx->rowbytes());
    if (e == hipSuccess) e = hipMalloc(&norms, (size_t)c * sizeof(float));
    for (int p = 0; p < 2; ++p) {
      if (e == hipSuccess && on[p] && (plane_oom >= 2 || (plane_oom == 1 && p == FILTER_BF16)))
        e = hipErrorOutOfMemory;
      if (e == hipSuccess && on[p]) e = hipMalloc(&fplane[p], (size_t)c * idx->planebytes(p));
      if (e == hipSuccess && on[p]) e = hipMalloc(&rn2[p], (size_t)c * sizeof(float));
    }
    if (e == hipSuccess && on[FILTER_I8])
      e = hipMalloc(&fscale, (size_t)c * sizeof(float));
    if (e == hipSuccess && on[FILTER_I8] && idx->l2aug())
      e = hipMalloc(&anorm, (size_t)c * sizeof(float));
    if (e == hipSuccess && on[FILTER_BF16] && idx->l2aug())
      e = hipMalloc(&anorm_b, (size_t)c * sizeof(float));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      release();
    }
    return e;
  };
  hipError_t e = allocate(cap);
  if (e != hipSuccess) scratch_trim(), e = allocate(cap);  // cached scratch chunks first
  if (e != hipSuccess) {  // retry without the growth headroom
    cap = need;
    e = allocate(cap);
  }
  // Still short of HBM: give up filter planes rather than rows (an fp32 inner-
  // product index holds 10 B per element with both planes, 7 with int8 only,
  // 4 without; searches then use the plane that remains, or the exact fp32
  // engine): bf16 first, then every plane.
  if (e != hipSuccess && on[FILTER_BF16] && on[FILTER_I8]) {
    on[FILTER_BF16] = false;
    e = allocate(cap);
  }
  if (e != hipSuccess && (on[FILTER_BF16] || on[FILTER_I8])) {
    on[FILTER_BF16] = on[FILTER_I8] = false;
    e = allocate(cap);
  }
  if (e != hipSuccess) return hip_fail(e, "vs: allocating row storage");
  const bool i8 = on[FILTER_I8];
  // zero every tail (tile reads past ntotal must see zeros, never NaN garbage)
  const int64_t keep = idx->ntotal;
  VS_HIP(hipMemsetAsync(codes + keep * idx->rowbytes(), 0, (size_t)(cap - keep) * idx->rowbytes(),
                        st),
         "vs: zeroing storage");
  VS_HIP(hipMemsetAsync(norms + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
         "vs: zeroing norms");
  for (int p = 0; p < 2; ++p) {
    if (!on[p]) continue;
    VS_HIP(hipMemsetAsync(rn2[p] + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
           "vs: zeroing residual norms");
  }
  if (i8)
    VS_HIP(hipMemsetAsync(fscale + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
           "vs: zeroing scales");
  if (anorm)
    VS_HIP(hipMemsetAsync(anorm + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
           "vs: zeroing augmented norms");
  if (anorm_b)
    VS_HIP(hipMemsetAsync(anorm_b + keep, 0, (size_t)(cap - keep) * sizeof(float), st),
           "vs: zeroing augmented norms");
  if (idx->codes && keep > 0) {
    VS_HIP(hipMemcpyAsync(codes, idx->codes, (size_t)keep * idx->rowbytes(),
                          hipMemcpyDeviceToDevice, st),
           "vs: copying storage");
    VS_HIP(hipMemcpyAsync(norms, idx->norms, (size_t)keep * sizeof(float),
                          hipMemcpyDeviceToDevice, st),
           "vs: copying norms");
    for (int p = 0; p < 2; ++p) {
      if (!on[p]) continue;
      // tile-major planes: rows [0, keep) are the first ceil(keep / 256) tiles
      VS_HIP(hipMemcpyAsync(fplane[p], idx->fplane[p],
                            (size_t)round_up(keep, 256) * idx->planebytes(p),
                            hipMemcpyDeviceToDevice, st),
             "vs: copying plane");
      VS_HIP(hipMemcpyAsync(rn2[p], idx->rn2[p], (size_t)keep * sizeof(float),
                            hipMemcpyDeviceToDevice, st),
             "vs: copying residual norms");
    }
    if (i8)
      VS_HIP(hipMemcpyAsync(fscale, idx->fscale, (size_t)keep * sizeof(float),
                            hipMemcpyDeviceToDevice, st),
             "vs: copying scales");
    if (anorm && idx->anorm)
      VS_HIP(hipMemcpyAsync(anorm, idx->anorm, (size_t)keep * sizeof(float),
                            hipMemcpyDeviceToDevice, st),
             "vs: copying augmented norms");
    if (anorm_b && idx->anorm_b)
      VS_HIP(hipMemcpyAsync(anorm_b, idx->anorm_b, (size_t)keep * sizeof(float),
                            hipMemcpyDeviceToDevice, st),
             "vs: copying augmented norms");
  }
  // the planes' rows past the kept ones read zeros (after the prefix copy,
  // which brings whole tiles)
  for (int p = 0; p < 2; ++p)
    if (on[p])
      VS_HIP(launch_plane_zero_rows(fplane[p], idx->planebytes(p), keep, cap - keep, st),
             "vs: zeroing plane");
  // The copies above, and searches of this index still in flight (any
  // stream), read the old storage; other indexes' work is not waited for.
  VS_HIP(hipStreamSynchronize(st), "vs: storage growth");
  VS_HIP(wait_readers(idx), "vs: storage growth");
  free_storage(idx);
  if (on[0] != idx->plane_on[0] || on[1] != idx->plane_on[1]) {
    // a plane lost to a memory shortage: said once on stderr and kept for
    // vs_notice (searches stay exact; the engines that remain are slower)
    char buf[256];
    snprintf(buf, sizeof(buf),
             "vsearch: HBM short at %lld rows: filter planes dropped (int8 %s, bf16 %s); "
             "searches use %s",
             (long long)cap, on[FILTER_I8] ? "kept" : "dropped",
             on[FILTER_BF16] ? "kept" : "dropped",
             on[FILTER_I8] || on[FILTER_BF16] ? "the remaining plane" : "the exact fp32 engine");
    idx->notice = buf;
    fprintf(stderr, "%s\n", buf);
  }
  idx->plane_on[0] = on[0];
  idx->plane_on[1] = on[1];
  idx->codes = codes;
  idx->norms = norms;
  for (int p = 0; p < 2; ++p) {
    idx->fplane[p] = fplane[p];
    idx->rn2[p] = rn2[p];
  }
  idx->fscale = fscale;
  idx->anorm = anorm;
  idx->anorm_b = anorm_b;
  idx->capacity = cap;
  return VS_OK;
}

void free_storage(vs_index* idx) {
  if (idx->codes) (void)hipFree(idx->codes);
  if (idx->norms) (void)hipFree(idx->norms);
  for (int p = 0; p < 2; ++p) {
    if (idx->fplane[p]) (void)hipFree(idx->fplane[p]);
    if (idx->rn2[p]) (void)hipFree(idx->rn2[p]);
    idx->fplane[p] = nullptr;
    idx->rn2[p] = nullptr;
  }
  if (idx->fscale) (void)hipFree(idx->fscale);
  if (idx->anorm) (void)hipFree(idx->anorm);
  if (idx->anorm_b) (void)hipFree(idx->anorm_b);
  idx->anorm_b = nullptr;
  idx->codes = nullptr;
  idx->norms = nullptr;
  idx->fscale = nullptr;
  idx->anorm = nullptr;
  idx->capacity = 0;
}

// What a search computes, shared by every engine.
struct SearchArgs {
  int mode = MODE_IP;
  const float* qbuf = nullptr;   // [nq_pad][ld] fp32 query rows (zero padded)
  const void* qb16 = nullptr;    // bf16 copy of the queries (bf16 indexes)
  const float* qaux = nullptr;   // |q|^2 (L2) or 1/|q| (COS), nq_pad entries
  const float* xaux = nullptr;   // per-row norms (L2) or 1/|x| (COS)
  int nq = 0, nq_pad = 0, k = 0;
  int64_t self0 = -1;            // self-join: query q is row self0 + q
  float min_score = 0.0f;
  int raw = 0;                   // VS_RAW_ORDER
  bool l2_direct = false;        // faiss's sequential branch (the call's nq < 20)
  // the call waits for its results anyway (host outputs): a small batch may
  // read its device-side count after the first stage and skip the empty rest
  bool host_wait = false;
  float* D = nullptr;
  int64_t* I = nullptr;
};

int run_topk(vs_index* idx, const SearchArgs& a, hipStream_t st, int force_engine);

// The exact engine on fp32 / bf16 rows: the fused MFMA GEMM + merge.  With
// qlist/qcount, the batch is the gathered queries qlist[0 .. *qcount)
// (device-side count) and the results go to their rows of D / I.
int run_gemm(vs_index* idx, const SearchArgs& a, int need, hipStream_t st,
              const int* qlist = nullptr, const int* qcount = nullptr) {
  const int KP = kp_for(need);
  const int ntotal = (int)idx->ntotal;
  Scratch scr(st);
  Partials part;
  part.KP = KP;
  const int nqt = a.nq_pad / kBQ;
  const int ntiles = (ntotal + kBN - 1) / kBN;
  // ~2 workgroups per CU on 256 CUs; never more splits than database tiles.
  // A gathered batch of unknown size spreads each query tile over the chip.
  const int nsplit = qlist ? (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, 256))
                           : (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, (512 + nqt - 1) / nqt));
  part.P = 2 * nsplit;
  const size_t n = (size_t)a.nq_pad * part.P * KP;
  VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
  const void* qmat = a.qb16 ? a.qb16 : (const void*)a.qbuf;
  {
    KernelTimer tm(st, qlist ? nullptr : "gemm_topk");
    VS_HIP(launch_gemm_topk(KP, a.mode, idx->codes, a.xaux, qmat, a.qaux, idx->ld, idx->esize,
                            ntotal, a.nq_pad, nsplit, a.self0, part, st, qlist, qcount),
           "vs: gemm_topk launch");
    tm.stop();
  }
  VS_HIP(launch_merge_partials(a.mode, part, qlist ? a.nq_pad : a.nq, a.k, idx->id_base,
                               a.min_score, a.D, a.I, a.k, st, a.raw, qlist, qcount),
         "vs: merge launch");
  return VS_OK;
}

int adaptive_record(vs_index* idx, const int* handed, int n, hipStream_t st);
int run_paged(vs_index* idx, const SearchArgs& a, hipStream_t st, const int* gl = nullptr,
              const int* gc = nullptr);
int run_gemm_rescored(vs_index* idx, const SearchArgs& a, int need, int KF, int plane,
                      hipStream_t st, const int* gl, const int* gc);

// The filter-and-verify engine (vs_gemm_x1.hip), entirely stream-ordered, as a
// chain of stages over the planes the index holds (int8, then bf16):
//  1. convert the stage's queries to its plane (int8 codes + scales, or bf16);
//     the x1 pass keeps 8-entry lane lists per query;
//  2. merge them to the KF best approximate candidates;
//  3. verify_rescore: exact keys of the candidates + the bound check (fail[]);
//  4. the flagged queries are compacted on the device and re-checked by the
//     wide verification (every lane-list entry below the list floors);
//  5. the merges emit (D, I) of the stage's queries;
//  6. the queries still flagged go to the next stage as a gathered batch
//     (device-side list and count: the int8 plane's wider bound leaves
//     clustered data to the bf16 plane), and after the last plane to the exact
//     fp32 engine (a launch whose tiles past the device-side count exit at
//     once), whose rows overwrite theirs.
// Counts live in device memory; the host reads one only to skip the later
// stages when none is left (tail_wait_on).  `gl` / `gc` (stages after the first): the batch is queries gl[0 .. *gc) of `a`.
// dump launches in the filter pass (default; env VS_X1_DUMP=0 runs every
// launch as a list launch, for A/B)
static bool dump_enabled() {
  static const bool v = [] {
    const char* e = getenv("VS_X1_DUMP");
    return !e || atoi(e) != 0;
  }();
  return v;
}

// Small batches through the staged engine's skinny passes (env
// VS_SMALL_FILTER=0 keeps the exact streaming kernels, for A/B; read at every
// search), over indexes of at least kSmallFilterMinRows rows.
constexpr int64_t kSmallFilterMinRows = 1 << 18;
bool small_filter_on() {
  const char* e = getenv("VS_SMALL_FILTER");
  return !e || atoi(e) != 0;
}
// L2 calls of fewer than 20 queries (faiss's sequential formula: the
// verification rescored with MODE_L2D) through the planes too (env
// VS_SMALL_L2D=0 keeps them on the exact GEMV, for A/B)
bool small_l2d_ok(int mode, const SearchArgs& a) {
  if (!(mode == MODE_L2 && a.l2_direct)) return true;
  const char* e = getenv("VS_SMALL_L2D");
  return !e || atoi(e) != 0;
}

// The deep stage's small-count kernel (env VS_SKINNY_DEEP=0 turns it off,
// for A/B; read at every search).
bool skinny_deep_on() {
  const char* e = getenv("VS_SKINNY_DEEP");
  return !e || atoi(e) != 0;
}

// Workgroups per filter-pass launch the database splits aim at: one round (256,
// one per CU) for batches of at most 8 query tiles, whose lane lists stay at
// 128+ per query (C2, 4 query tiles: 256 lists, 405-407k -> 436-441k
// queries/s, profiles/r06wgs); two rounds (512) above, where one round would
// cut the lists to 64 per query and saturate some (the 1.25M-row rank of an
// 8-GPU C3: 11 queries per search to the deep stage, 441k -> 423k).  Env
// VS_X1_WGS overrides (A/B; read at every search).
static int x1_wg_target(int nqt) {
  const char* e = getenv("VS_X1_WGS");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : nqt <= 8 ? 256 : 512;
}

// Whether a search reads the count of queries a stage leaves flagged (a 4-byte
// copy to pinned memory and a wait on the stream) and enqueues the later stages
// only when some remain.  Host-output calls wait for their results anyway;
// device-output calls wait too: the later stages over an empty count are ~45
// launches of ~5 us each (0.25 ms of a 2.39-ms C2 search, 0.58 ms of the
// 1.25M-row rank's 10.5 ms, profiles/r06tl), far more than the wait.  Not on a
// capturing stream (a graph keeps every launch).  Env VS_TAIL_WAIT=0 keeps
// every launch (A/B; read at every search).
static bool tail_wait_on(const SearchArgs& a, hipStream_t st) {
  const char* e = getenv("VS_TAIL_WAIT");
  if (e && atoi(e) == 0) return false;
  if (a.host_wait) return true;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return cs == hipStreamCaptureStatusNone;
}

// The device-side count *dcount once the stream has reached this point (one
// pinned int per host thread).
static int read_count(const int* dcount, hipStream_t st, int* out) {
  static thread_local int* pin = nullptr;
  if (!pin) VS_HIP(hipHostMalloc((void**)&pin, sizeof(int), hipHostMallocPortable), "vs: count");
  VS_HIP(hipMemcpyAsync(pin, dcount, sizeof(int), hipMemcpyDeviceToHost, st), "vs: count");
  VS_HIP(hipStreamSynchronize(st), "vs: count");
  *out = *pin;
  return VS_OK;
}

int run_filter_verify(vs_index* idx, const SearchArgs& a, int need, int KF, hipStream_t st,
                      int plane, bool last_plane, bool deep = false, const int* gl = nullptr,
                      const int* gc = nullptr) {
  const int ntotal = (int)idx->ntotal;
  const int mode = a.mode;
  const bool gathered = gl != nullptr;
  Scratch scr(st);
  X1Args x;
  x.nq_pad = (int)round_up(a.nq_pad, kX1Q);
  const int nq = gathered ? x.nq_pad : a.nq;  // slots of this stage
  const int nqt = x.nq_pad / kX1Q;
  const int ntiles = (ntotal + kX1Q - 1) / kX1Q;
  const int L = x1_lane_len();
  // enough lists that their 4*nsplit*L entries cover 16*KF candidates (C4's
  // self-join, KF = 64: 128 lists, which lets the int8 stage settle it: 283k ->
  // 372k students/s, profiles/r02zc), and the workgroup target (x1_wg_target:
  // two per CU on 256 CUs at C3, 128 lists per query; one per CU up to 8 query
  // tiles).  More lists put the wide check's floor T (the best last entry of a
  // full list) deeper behind the top-M, which the bound needs on clustered data
  // and on the int8 plane (profiles/r02l_ab_split.txt; one workgroup per CU left
  // 0.7 % of the C3 queries to the exact engine on int8)
  // Inner product past k = 32 (M = 2k - 1 of 59 .. 127, KF = 64 / 128) takes
  // twice as many lists again: at C3 (B = 4096) k = 30 left 13 queries per
  // search and k = 60 815 to the deep bf16 stage (a 10M-row pass of ~20-30 ms
  // however few they are); with 8 KF / L lists 0 and 26 (60.5 vs 78.9 and 85.9
  // vs 94.2 ms per search, profiles/r05q, VS_X1_SPLIT_MULT=2)
  const int lists_per_cand = mode == MODE_IP && KF >= 64 ? 8 : 4;
  const int wg_target = x1_wg_target(nqt);
  x.nsplit = (int)std::max<int64_t>(
      std::min<int64_t>(ntiles, lists_per_cand * ((KF + L - 1) / L)),
      std::min<int64_t>(ntiles, (wg_target + nqt - 1) / nqt));
  // the deep stage (a gathered batch of the few queries an earlier stage could
  // not settle): as many lists as two workgroups per CU give ONE query tile, so
  // the floors sit far behind the top (the a_M + 2B threshold keeps the wide
  // set small)
  // (lane lists of at most ~1 GB: x.nq_pad slots x 4 nsplit lists x 8 entries x 8 B)
  if (deep)
    x.nsplit = (int)std::max<int64_t>(
        x.nsplit, std::min<int64_t>({ntiles, 512, (1ll << 30) / ((int64_t)x.nq_pad * 4 * 8 * 8)}));
  // A first pass on the bf16 plane (the adaptive order's choice when int8
  // hands on too many: embedding-like clustered rows) takes twice the lists:
  // its checks then settle more queries and fewer go to the deep stage
  // (clustered C3 37.1k -> 43.0k queries/s; on uniform rows the int8 pass
  // loses 3 % with them; profiles/r05s)
  if (!gathered && !deep && plane == FILTER_BF16)
    x.nsplit = (int)std::min<int64_t>(ntiles, 2 * (int64_t)x.nsplit);
  // A small batch (at most skinny_plane_max_queries() queries, the first stage
  // of a search routed here by run_topk) streams its plane once through
  // skinny_plane_topk instead of an x1 pass over a whole query tile: 2,048
  // lists of 8 per query, the deep stage's count
  const bool small = !gathered && !deep && a.nq <= skinny_plane_max_queries() && a.self0 < 0 &&
                     (mode == MODE_IP || (mode == MODE_L2 && idx->l2aug()));  // the pass's IP
  if (small) x.nsplit = (int)std::min<int64_t>(512, std::max<int64_t>(1, (ntiles + 3) / 4));
  x.nsplit = std::max(x.nsplit, 1);
  {  // A/B: more (shorter) database splits = more lane lists per query
    static const int mult = [] {
      const char* e = getenv("VS_X1_SPLIT_MULT");
      return e && atoi(e) > 1 ? atoi(e) : 1;
    }();
    x.nsplit = (int)std::min<int64_t>(ntiles, (int64_t)x.nsplit * mult);
  }
  Partials part;  // lane lists: L entries each
  part.KP = L;
  part.P = 4 * x.nsplit;
  const size_t np_ = (size_t)x.nq_pad * part.P * part.KP;
  VS_HIP(scr.alloc((void**)&part.key, np_ * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&part.id, np_ * sizeof(int)), "vs: scratch");
  // this stage's fp32 query rows and aux values: the staged batch, the stored
  // rows (self-joins), or a gathered copy of the flagged ones
  const float* Q = a.self0 >= 0 ? (const float*)idx->row(a.self0) : a.qbuf;
  const float* qaux = a.qaux;
  int* qrow = nullptr;
  if (gathered) {
    float *qc = nullptr, *ac = nullptr;
    VS_HIP(scr.alloc((void**)&qc, (size_t)x.nq_pad * idx->ld * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&ac, (size_t)x.nq_pad * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&qrow, (size_t)x.nq_pad * sizeof(int)), "vs: scratch");
    VS_HIP(launch_gather_queries(Q, idx->ld, a.qaux, gl, gc, x.nq_pad, a.self0, qc, ac, qrow, st),
           "vs: gathered queries");
    Q = qc;
    qaux = ac;
  }
  const bool self_rows = a.self0 >= 0 && !gathered;  // queries are stored rows in place
  const int qa_rows = gathered ? x.nq_pad : a.nq_pad;  // rows of Q / qaux
  // query plane: a conversion of the stage's queries, or the stored rows' plane
  const bool i8 = plane == FILTER_I8;
  // L2: the pass is the inner product of the augmented rows and queries
  // (vs_index::aug_m, either plane); its lists are mapped to L2 keys after it
  const bool aug = mode == MODE_L2 && idx->l2aug();
  if (aug && (idx->aug_m <= 0 || self_rows)) return fail(VS_E_INVALID, "vs: int8 L2 plane");
  const int kmode = aug ? MODE_IP : mode;  // the pass's own metric
  // the verification's exact keys: an L2 call of fewer than 20 queries takes
  // faiss's sequential formula (the rounded exact sum of (x - q)^2), larger
  // ones its BLAS formula
  const int vmode = mode == MODE_L2 && a.l2_direct ? MODE_L2D : mode;
  const int64_t pb = idx->planebytes(plane);
  const char* QH = nullptr;
  const float* qs = nullptr;    // int8: query scales
  const float* qr2 = nullptr;   // int8: query residual norms (for the bound)
  // stored rows starting on a tile boundary are read from the index's own
  // (tile-major) plane; any other batch is converted (the same codes)
  const bool plane_rows = self_rows && a.self0 % kX1Q == 0;
  x.qtile0 = plane_rows ? (int)(a.self0 / kX1Q) : 0;
  if (plane_rows) {
    QH = idx->fplane[plane];
    if (i8) {
      qs = idx->fscale + a.self0;
      qr2 = idx->rn2[FILTER_I8] + a.self0;
    }
  } else {
    char* qh = nullptr;
    VS_HIP(scr.alloc((void**)&qh, (size_t)x.nq_pad * pb), "vs: scratch");
    if (i8) {
      float *sc = nullptr, *r = nullptr;
      VS_HIP(scr.alloc((void**)&sc, (size_t)qa_rows * sizeof(float)), "vs: scratch");
      VS_HIP(scr.alloc((void**)&r, (size_t)qa_rows * sizeof(float)), "vs: scratch");
      if (aug)
        VS_HIP(launch_quantize_i8_l2aug(Q, idx->ld, 0, qa_rows, idx->aug, nullptr, (int8_t*)qh, sc,
                                        r, nullptr, st),
               "vs: query plane");
      else
        VS_HIP(launch_quantize_i8(Q, idx->ld, 0, qa_rows, (int8_t*)qh, sc, r, st),
               "vs: query plane");
      qs = sc;
      qr2 = r;
    } else if (aug) {
      VS_HIP(launch_bf16_plane_l2aug(Q, idx->ld, 0, qa_rows, idx->aug, nullptr, (uint16_t*)qh,
                                     nullptr, nullptr, st),
             "vs: query plane");
    } else {
      VS_HIP(launch_bf16_plane(Q, idx->ld, 0, qa_rows, (uint16_t*)qh, st), "vs: query plane");
    }
    VS_HIP(launch_plane_zero_rows(qh, pb, qa_rows, x.nq_pad - qa_rows, st), "vs: query plane");
    QH = qh;
  }
  const unsigned* stats = idx->bstats[plane];  // the index's maxima (kept by add / remove)
  x.filter = plane;
  x.XH = idx->fplane[plane];
  x.xs = idx->fscale;
  if (i8 && mode == MODE_COS) {
    // the cosine folds the inverse norms into the int8 factors: s_x / |x| per
    // row (capacity rows: tiles read past ntotal), s_q / |q| per query
    float* cx = nullptr;
    VS_HIP(scr.alloc((void**)&cx, (size_t)idx->capacity * sizeof(float)), "vs: scratch");
    VS_HIP(launch_mul_arrays(idx->fscale, a.xaux, idx->capacity, cx, st), "vs: cosine factors");
    x.xs = cx;
    if (plane_rows) {
      qs = cx + a.self0;
    } else {
      float* cq = nullptr;
      VS_HIP(scr.alloc((void**)&cq, (size_t)qa_rows * sizeof(float)), "vs: scratch");
      VS_HIP(launch_mul_arrays(qs, qaux, qa_rows, cq, st), "vs: cosine factors");
      qs = cq;
    }
  }
  if (i8) {  // the per-lane factor bounds of the fast reject (scalar loads in the kernel)
    float* gm = nullptr;
    const size_t ng = (size_t)(idx->capacity / 16);
    VS_HIP(scr.alloc((void**)&gm, 2 * ng * sizeof(float)), "vs: scratch");
    VS_HIP(launch_group_max(x.xs, idx->capacity, gm, st, ntotal, gm + ng), "vs: factor bounds");
    x.xgmax = gm;
    x.xgmin = gm + ng;
  }
  x.xaux = a.xaux;
  x.QH = QH;
  x.qs = qs;
  x.qaux = qaux;
  x.nqa = qa_rows;
  x.ld = !aug ? idx->ld : i8 ? idx->ld + idx->aug_m : idx->ld + kAugBf16;  // the plane's K
  x.ntotal = ntotal;
  x.self0 = self_rows ? a.self0 : -1;
  x.qrow = qrow;
  x.qcount = gc;
  const BoundArgs ba = aug ? make_bound_args_l2aug(idx->ld, idx->aug, plane)
                           : make_bound_args(idx->ld, plane);
  if (!gathered && !small && x1_dump_applies(kmode, plane) && dump_enabled() &&
      x1_pass_dumps(ntotal, x.nsplit)) {
    // query cuts + dump launches (vs_gemm_x1.hip header and "Query cuts"): the
    // cuts are set after the pass's first launch and are the verification's
    // floor for the rows the dump launches drop.  The dump slots: up to
    // x1_dump_slots() candidate rows per lane list and segment within ~4 GB;
    // fewer than 16 (or no memory): every launch is a list launch.
    const int64_t lists = (int64_t)x.nq_pad * part.P;
    const int dR = (int)std::min<int64_t>(x1_dump_slots(), (int64_t(4) << 30) / (lists * 8));
    if (dR >= 16) {
      int *dc = nullptr, *ds = nullptr;
      hipError_t e = scr.alloc((void**)&dc, (size_t)lists * sizeof(int));
      if (e == hipSuccess) e = scr.alloc((void**)&ds, (size_t)lists * dR * 2 * sizeof(int));
      if (e == hipSuccess) {
        VS_HIP(scr.alloc((void**)&x.qcut, (size_t)qa_rows * sizeof(float)), "vs: scratch");
        double* bk = nullptr;
        VS_HIP(scr.alloc((void**)&bk, (size_t)qa_rows * sizeof(double)), "vs: scratch");
        VS_HIP(hipMemsetD32Async((hipDeviceptr_t)x.qcut, 0x7f7fffff, (size_t)qa_rows, st),
               "vs: cuts");
        VS_HIP(hipMemsetAsync(dc, 0, (size_t)lists * sizeof(int), st), "vs: dumps");
        VS_HIP(launch_qbound(mode, Q, idx->ld, qaux, plane, stats, qr2, qa_rows, bk, st, &ba),
               "vs: cuts");
        x.qbkey = bk;
        x.qcut_m = need;
        x.dump = true;
        x.dcount = dc;
        x.dslot = ds;
        x.dR = dR;
        x.dstats = device_stats(idx->device) ? device_stats(idx->device) + 6 : nullptr;
      } else {
        (void)hipGetLastError();  // out of memory for the dumps: list launches
      }
    }
  }
  {
    // the pass as a whole (list + dump launches and the cut / replay kernels
    // between them) under "<name>_pass", beside the per-launch spans
    KernelTimer whole(st, gathered ? nullptr : i8 ? "gemm_topk_x1_i8_pass" : "gemm_topk_x1_pass",
                      false);
    X1SpanTimer tm(i8 ? "gemm_topk_x1_i8" : "gemm_topk_x1",
                   i8 ? "gemm_topk_x1_i8_list" : "gemm_topk_x1_list");
    if (!gathered) x.timing = &tm;
    // the deep bf16 stage of a few queries (inner product / augmented L2, not
    // a self-join): skinny_plane_topk streams the plane once for them and
    // the x1 pass exits, or the reverse, by the device-side count
    if (gathered && deep && !i8 && kmode == MODE_IP && a.self0 < 0 && skinny_deep_on()) {
      VS_HIP(launch_skinny_plane(FILTER_BF16, x.XH, x.QH, x.ld, ntotal, gc, nullptr, nullptr, part,
                                 st),
             "vs: skinny deep stage");
      x.qskip = skinny_plane_max_queries();
    }
    if (small) {
      int* cnt = nullptr;
      VS_HIP(scr.alloc((void**)&cnt, sizeof(int)), "vs: scratch");
      VS_HIP(hipMemsetD32Async((hipDeviceptr_t)cnt, a.nq, 1, st), "vs: count");
      KernelTimer ks(st, i8 ? "skinny_plane_topk_i8" : "skinny_plane_topk");
      VS_HIP(launch_skinny_plane(plane, x.XH, x.QH, x.ld, ntotal, cnt, qs, x.xs, part, st, a.nq),
             "vs: skinny first stage");
      ks.stop();
    } else {
      int nd = 0;
      VS_HIP(launch_gemm_topk_x1(kmode, x, part, st, &nd), "vs: gemm_topk_x1 launch");
    }
    x.timing = nullptr;
    whole.stop();
  }
  if (aug)  // augmented inner-product keys A -> L2 keys |q|^2 + 2A (lists and cuts)
    VS_HIP(launch_l2aug_map(part.key, part.id, (int64_t)part.P * part.KP, qa_rows, qaux,
                            idx->aug.nref, x.qcut, st),
           "vs: L2 keys");

  // approximate top-KF per query (plain lexicographic order: the L2 merge)
  float* Dk = nullptr;
  int64_t* Ik = nullptr;
  VS_HIP(scr.alloc((void**)&Dk, (size_t)nq * KF * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&Ik, (size_t)nq * KF * sizeof(int64_t)), "vs: scratch");
  if (KF > 64) {  // 2k - 1 > 64 (inner product, k > 32): the select kernel
    VS_HIP(launch_select_lists(part, L, nq, KF, Dk, Ik, st, gc), "vs: merge");
  } else if (select_heads_applies(part, L, KF)) {
    VS_HIP(launch_select_heads(part, nq, KF, Dk, Ik, st, gc), "vs: merge");
  } else {
    Partials mp = part;
    mp.KP = kp_for(KF);
    mp.KL = L;
    VS_HIP(launch_merge_partials(MODE_L2, mp, nq, KF, 0, 0.0f, Dk, Ik, KF, st, 0, nullptr, gc),
           "vs: merge");
  }
  Partials vp;
  vp.KP = kp_for(KF);
  vp.P = 1;
  int* flags = nullptr;
  int* qlist = nullptr;
  int* qcount = nullptr;
  VS_HIP(scr.alloc((void**)&vp.key, (size_t)nq * vp.KP * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&vp.id, (size_t)nq * vp.KP * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&flags, (size_t)nq * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&qlist, (size_t)x.nq_pad * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&qcount, 2 * sizeof(int)), "vs: scratch");
  const float* qinv = mode == MODE_COS ? qaux : nullptr;
  const float* xinv = mode == MODE_COS ? a.xaux : nullptr;
  VS_HIP(launch_verify_rescore(vmode, nq, KF, need, Dk, Ik, idx->codes, idx->norms, Q, qaux,
                               idx->ld, ba, stats, part, L, vp.key, vp.id, vp.KP, flags, st, qinv,
                               xinv, qr2, gc, x.qcut, idx->esize),
         "vs: verify");
  unsigned long long* dst = device_stats(idx->device);
  if (!dst) return fail(VS_E_HIP, "vs: statistics buffer");
  // statistics: [0] queries (first stage), [1] flagged by a first check, [2]
  // redone by the exact engine, [3] handed to a second filter stage
  VS_HIP(launch_compact_flags(flags, nq, qlist, qcount, dst + 1, gathered ? nullptr : dst + 0, st),
         "vs: flags");
  if (wide_enabled())
    VS_HIP(launch_verify_wide(vmode, nq, qlist, qcount, KF, need, idx->codes, idx->norms, Q, qaux,
                              idx->ld, ba, stats, part, L, vp.key, vp.id, vp.KP, flags, st, qinv,
                              xinv, qr2, Dk, Ik, dst + 4, x.qcut, idx->esize),
           "vs: verify wide");
  VS_HIP(launch_compact_flags(flags, nq, qlist, qcount + 1, last_plane ? dst + 2 : dst + 3,
                              nullptr, st),
         "vs: flags");
  VS_HIP(launch_merge_partials(vmode, vp, nq, a.k, idx->id_base, a.min_score, a.D, a.I, a.k, st,
                               a.raw, gl, gc),
         "vs: merge");
  // The first stage's and the deep stage's leftovers, read when the call may
  // wait (tail_wait_on): nothing left, no later stage is enqueued (the live
  // search_catalog path, mcp_book_server.py:142, at batch 1: ~30 launches,
  // 0.13 ms of a 2.6-ms search; C2 ~45, 0.25 ms)
  if ((!gathered || deep) && tail_wait_on(a, st)) {
    int left = -1;
    int rc = read_count(qcount + 1, st, &left);
    if (rc) return rc;
    if (left == 0) {
      if (!last_plane && !gathered && plane == FILTER_I8) {
        rc = adaptive_record(idx, qcount + 1, nq, st);
        if (rc) return rc;
      }
      return VS_OK;
    }
  }
  // what is still flagged (usually nothing: every tile exits), as query ids of `a`
  const int* next = qlist;
  if (gathered) {
    int* composed = nullptr;
    VS_HIP(scr.alloc((void**)&composed, (size_t)x.nq_pad * sizeof(int)), "vs: scratch");
    VS_HIP(launch_compose_list(gl, qlist, qcount + 1, x.nq_pad, composed, st), "vs: flags");
    next = composed;
  }
  if (!last_plane) {
    if (!gathered && plane == FILTER_I8) {
      int rc = adaptive_record(idx, qcount + 1, nq, st);
      if (rc) return rc;
    }
    return run_filter_verify(idx, a, need, KF, st, FILTER_BF16, true, true, next, qcount + 1);
  }
  // the exact redo (untimed: the kernel timer holds the first filter pass)
  return run_gemm_rescored(idx, a, need, KF, plane, st, next, qcount + 1);
}

// The staged engine's last stage: the exact fp32 MFMA GEMM (bf16 rows: the
// bf16 one) over the queries no filter stage settled (gathered: gl[0 .. *gc) of
// `a`) keeps KF candidates per query, which are rescored like every other
// stage's (verify_rescore: fp64 sums, one rounding), so every key the staged
// engine returns is the fp32 rounding of the exact score (oracle/flat.py
// key_window); the candidates are proven with the GEMM's own bound and what it
// cannot prove goes to the exact-key stream (below).
// Slots of the exact-key stream per launch (its lists: kExactSlots x up to
// 256 row blocks x KP entries); launches past the device-side count exit.
constexpr int kExactSlots = 256;
constexpr int kXPageSlots = 1024;  // run_paged's exact-key pages
bool exact_stream_on() {
  const char* e = getenv("VS_EXACT_STREAM");
  return !e || atoi(e) != 0;
}

int run_gemm_rescored(vs_index* idx, const SearchArgs& a, int need, int KF, int plane,
                      hipStream_t st, const int* gl, const int* gc) {
  // more than the 64 entries one exact page holds (inner product, k > 32): the
  // paged exact engine over the gathered queries (its keys are the fp32
  // engine's own, as in a search that never went through the filter)
  if (KF > 64) return run_paged(idx, a, st, gl, gc);
  const int ntotal = (int)idx->ntotal;
  const int KP = kp_for(KF);
  const int nslot = (int)round_up(a.nq, kBQ);
  Partials part;
  part.KP = KP;
  const int ntiles = (ntotal + kBN - 1) / kBN;
  const int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, 256));
  part.P = 2 * nsplit;
  // The gathered queries run in slot windows of at most `cap` slots, so the
  // lists stay within ~1 GB whatever the batch (a 65,536-student self-join
  // chunk at KP = 64 would need 16 GB for every slot at once); windows past
  // the device-side count exit at once (usually all but the first).
  const int cap = (int)std::min<int64_t>(
      nslot, std::max<int64_t>(kBQ, ((int64_t)1 << 30) / ((int64_t)part.P * KP * 8) / kBQ * kBQ));
  Scratch scr(st);
  const size_t n = (size_t)cap * part.P * KP;
  VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
  float *qc = nullptr, *ac = nullptr;
  int* qrow = nullptr;
  VS_HIP(scr.alloc((void**)&qc, (size_t)cap * idx->ld * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&ac, (size_t)cap * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&qrow, (size_t)cap * sizeof(int)), "vs: scratch");
  float* Dk = nullptr;
  int64_t* Ik = nullptr;
  VS_HIP(scr.alloc((void**)&Dk, (size_t)cap * KF * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&Ik, (size_t)cap * KF * sizeof(int64_t)), "vs: scratch");
  Partials vp;
  vp.KP = KP;
  vp.P = 1;
  int* flags = nullptr;
  int* wc = nullptr;
  VS_HIP(scr.alloc((void**)&vp.key, (size_t)cap * KP * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&vp.id, (size_t)cap * KP * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&flags, (size_t)cap * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&wc, sizeof(int)), "vs: scratch");
  const float* Qa = a.self0 >= 0 ? (const float*)idx->row(a.self0) : a.qbuf;
  uint16_t* qc16 = nullptr;
  if (idx->esize == 2) {
    if (a.self0 >= 0 || !a.qb16) return fail(VS_E_INVALID, "vs: bf16 last stage");
    VS_HIP(scr.alloc((void**)&qc16, (size_t)cap * idx->ld * sizeof(uint16_t)), "vs: scratch");
  }
  const float* qinv = a.mode == MODE_COS ? ac : nullptr;
  const float* xinv = a.mode == MODE_COS ? a.xaux : nullptr;
  const int emode = a.mode == MODE_L2 && a.l2_direct ? MODE_L2D : a.mode;
  // The candidates are proven with the fp32 GEMM's own error bound (no plane
  // residuals: BoundArgs::rows_exact); a query it cannot settle (more than
  // KF - k rows inside the bound of its k-th: dense near-ties) is ranked over
  // every row by its exact key instead (vs_exact.hip; env VS_EXACT_STREAM=0
  // keeps the fp32 candidates, for A/B), so every answer of the staged engine
  // is the exact top-k of the rescored keys.
  BoundArgs ba = make_bound_args(idx->ld, FILTER_BF16);
  ba.rows_exact = 1;
  const bool stream_ok =
      exact_stream_on() && idx->esize == 4 && exact_stream_nq(idx->ld) > 0 && KP <= 64;
  unsigned long long* dstats = device_stats(idx->device);
  int *fl = nullptr, *fc = nullptr, *ol = nullptr, *ewc = nullptr;
  int xslots = kExactSlots;
  Partials ep;
  if (stream_ok) {
    VS_HIP(scr.alloc((void**)&fl, (size_t)cap * sizeof(int)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&fc, sizeof(int)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&ol, (size_t)cap * sizeof(int)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&ewc, sizeof(int)), "vs: scratch");
    ep.KP = kp_for(need);
    ep.P = (int)std::min<int64_t>(256, std::max<int64_t>(1, ((int64_t)ntotal + 1023) / 1024));
    // slots per launch: the whole window when its lists fit in ~256 MB (C3:
    // one launch triple over an empty count instead of 16), else kExactSlots
    xslots = (int)std::min<int64_t>(
        cap, std::max<int64_t>(kExactSlots, ((int64_t)256 << 20) / ((int64_t)ep.P * ep.KP * 8)));
    VS_HIP(scr.alloc((void**)&ep.key, (size_t)xslots * ep.P * ep.KP * sizeof(float)),
           "vs: scratch");
    VS_HIP(scr.alloc((void**)&ep.id, (size_t)xslots * ep.P * ep.KP * sizeof(int)),
           "vs: scratch");
  }
  // A small batch (its flagged queries are at most its a.nq <= kSkinnyMaxQ):
  // the skinny fp32 kernel streams the rows once over the gathered queries
  // (slots past the device-side count score garbage that no merge reads)
  // instead of a GEMM over a whole query tile
  const bool skinny = a.nq <= kSkinnyMaxQ && KP <= 32 && (a.nq <= 16 || KP <= 16) && a.self0 < 0 &&
                      (a.mode == MODE_IP || a.mode == MODE_L2) && (idx->ld * idx->esize) % 128 == 0;
  Partials sp;
  if (skinny) {
    sp.KP = KP;
    sp.P = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (ntotal + 255) / 256));
    VS_HIP(scr.alloc((void**)&sp.key, (size_t)kSkinnyMaxQ * sp.P * KP * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&sp.id, (size_t)kSkinnyMaxQ * sp.P * KP * sizeof(int)), "vs: scratch");
  }
  for (int w0 = 0; w0 < nslot; w0 += cap) {
    const int* wl = gl + w0;  // this window's query ids, wc[0] of them
    VS_HIP(launch_window_count(gc, w0, cap, wc, st), "vs: window");
    // the window's query rows and aux values, slot by slot, for the rescoring
    VS_HIP(launch_gather_queries(Qa, idx->ld, a.qaux, wl, wc, cap, a.self0, qc, ac, qrow, st),
           "vs: gathered queries");
    // bf16 rows: the bf16 kernels take bf16 query rows (the staged values are
    // already bf16-rounded, so the conversion is exact)
    if (qc16) VS_HIP(launch_f32_to_bf16(qc, idx->ld, qc16, idx->ld, cap, idx->ld, st), "vs: bf16 queries");
    if (skinny) {
      VS_HIP(launch_skinny_topk(KP, a.mode, a.nq, idx->codes, idx->esize, a.xaux,
                                qc16 ? (const void*)qc16 : (const void*)qc, ac, idx->ld, ntotal,
                                sp.P, sp, st, wc),
             "vs: skinny_topk launch");
    } else {
      VS_HIP(launch_gemm_topk(KP, a.mode, idx->codes, a.xaux,
                              idx->esize == 2 ? a.qb16 : (const void*)Qa, a.qaux, idx->ld,
                              idx->esize, ntotal, cap, nsplit, a.self0, part, st, wl, wc),
             "vs: gemm_topk launch");
    }
    VS_HIP(launch_merge_partials(MODE_L2, skinny ? sp : part, skinny ? a.nq : cap, KF, 0, 0.0f, Dk,
                                 Ik, KF, st, 0, nullptr, wc),
           "vs: merge");
    VS_HIP(launch_verify_rescore(emode, cap, KF, need, Dk, Ik, idx->codes, idx->norms, qc, ac,
                                 idx->ld, ba, idx->bstats[plane], skinny ? sp : part, KP, vp.key,
                                 vp.id, vp.KP, flags, st, qinv, xinv, nullptr, wc, nullptr,
                                 idx->esize),
           "vs: rescore");
    VS_HIP(launch_merge_partials(emode, vp, cap, a.k, idx->id_base, a.min_score, a.D, a.I, a.k,
                                 st, a.raw, wl, wc),
           "vs: merge");
    if (!stream_ok) continue;
    // the queries the fp32 bound leaves open: every row ranked by its exact key
    VS_HIP(launch_compact_flags(flags, cap, fl, fc, dstats ? dstats + 8 : nullptr, nullptr, st),
           "vs: exact stream");
    VS_HIP(launch_compose_list(wl, fl, fc, cap, ol, st), "vs: exact stream");
    ExactStreamArgs ea;
    ea.X = (const float*)idx->codes;
    ea.xn = idx->norms;
    ea.xinv = xinv;
    ea.ld = idx->ld;
    ea.ntotal = ntotal;
    ea.Q = qc;
    ea.qaux = ac;
    ea.qrow = a.self0 >= 0 ? qrow : nullptr;
    ea.slots = fl;
    ea.count = fc;
    ea.nslot = xslots;
    for (int s0 = 0; s0 < cap; s0 += xslots) {
      ea.s0 = s0;
      VS_HIP(launch_window_count(fc, s0, xslots, ewc, st), "vs: exact stream");
      VS_HIP(launch_exact_stream(ep.KP, emode, ea, ep, st), "vs: exact stream");
      VS_HIP(launch_merge_partials(emode, ep, xslots, a.k, idx->id_base, a.min_score, a.D,
                                   a.I, a.k, st, a.raw, ol + s0, ewc),
             "vs: merge");
    }
  }
  return VS_OK;
}

// Fraction of int8-stage queries handed on to bf16 above which the int8 stage
// costs more than it saves (stage costs ~0.58 and 1 of a bf16-only search:
// break-even ~0.42).
constexpr double kI8HandOffMax = 0.3;

// Whether this search starts on the int8 plane (see vs_index::Adaptive).  While
// the int8 stage hands on too much, searches start on bf16, with an int8 probe
// after 8, 16, 32, 64 of them (each probe's counters arrive with a later
// search; a probe on clustered data costs ~1.4x a bf16-first search).
bool adaptive_use_i8(vs_index* idx) {
  auto& A = idx->ad;
  std::lock_guard<std::mutex> g(A.mu);
  bool fresh = false;
  if (A.pending && hipEventQuery(A.ev) == hipSuccess) {
    const unsigned long long q = A.hmirror[0], h = A.hmirror[1];
    if (q > A.seen_q) {
      const double f = (double)(h - A.seen_h) / (double)(q - A.seen_q);
      A.ema = A.have ? 0.5 * A.ema + 0.5 * f : f;
      A.have = true;
      fresh = true;
    }
    A.seen_q = q;
    A.seen_h = h;
    A.pending = false;
  }
  if (!A.have || A.ema <= kI8HandOffMax) {
    A.backoff = kI8FirstBackoff;
    A.skip_left = 0;
    return true;
  }
  if (fresh) {
    A.skip_left = A.backoff;
    A.backoff = std::min(2 * A.backoff, kI8MaxBackoff);
  }
  if (A.skip_left > 0) {
    --A.skip_left;
    return false;
  }
  A.skip_left = A.backoff;  // a probe; bf16 until its counters arrive
  return true;
}

// The per-index counters of an int8-first search: what the int8 stage saw
// and handed on, then an async copy to the pinned mirror (one in flight).
int adaptive_record(vs_index* idx, const int* handed, int n, hipStream_t st) {
  auto& A = idx->ad;
  std::lock_guard<std::mutex> g(A.mu);
  if (!A.dcount) {
    VS_HIP(hipMalloc(&A.dcount, 2 * sizeof(unsigned long long)), "vs: adaptive counters");
    VS_HIP(hipMemset(A.dcount, 0, 2 * sizeof(unsigned long long)), "vs: adaptive counters");
    VS_HIP(hipHostMalloc(&A.hmirror, 2 * sizeof(unsigned long long)), "vs: adaptive counters");
    A.hmirror[0] = A.hmirror[1] = 0;
    VS_HIP(hipEventCreateWithFlags(&A.ev, hipEventDisableTiming), "vs: adaptive counters");
  }
  VS_HIP(launch_add_counts(handed, n, A.dcount, st), "vs: adaptive counters");
  if (!A.pending) {
    VS_HIP(hipMemcpyAsync(A.hmirror, A.dcount, 2 * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, st),
           "vs: adaptive counters");
    VS_HIP(hipEventRecord(A.ev, st), "vs: adaptive counters");
    A.pending = true;
  }
  return VS_OK;
}

// The paged exact engine: any k, every metric, for what one 64-entry list
// cannot answer — k > 64, raw (shard) lists past 64, and faiss's inner-product
// tie rule past k = 32 (it reads the k-th key's run of equal keys up to 2k - 1
// entries; service.py:529-531 oversamples to k = 60, and the live tool's k is
// the agent's, mcp_book_server.py:115,142).  faiss's IndexFlat::search has no k
// limit; neither has this.  A query's answer is read off its lexicographic
// (key, row) order in pages of 64 entries:
//  1. page 1: the exact kernel's top-64 (FLOOR form with the floor (-inf, -1));
//  2. page_step: a query takes page p + 1 only while its answer needs it (fewer
//     than k entries so far, or the rule's run of k-th key ties reaching the
//     page's end below 2k - 1) and its page came back full; page p + 1 = the
//     same kernel with the admission floored at page p's last entry, over the
//     queries that need it (gathered on the device; launches past the count
//     exit at once), so every row's key is the same instructions' result in
//     every page;
//  3. page_finish: the pages side by side, faiss's rule (unless raw or not
//     inner product), the k outputs (empty past the rows there are).
// Kernels: the fp32 GEMV for one or two fp32 inner-product queries and for
// faiss's sequential L2 branch (calls under 20 queries, groups of up to 8);
// everything else the fp32 / bf16 MFMA GEMM (self-joins included).  Query
// windows keep the pages within ~2 GB whatever k and the batch.
// gl / gc: a gathered batch, queries gl[0 .. *gc) of `a` (the staged engine's
// last stage for inner product k > 32; device-side count), whose rows alone
// are written.
int run_paged(vs_index* idx, const SearchArgs& a, hipStream_t st, const int* gl, const int* gc) {
  const bool gathered = gl != nullptr;
  const int ntotal = (int)idx->ntotal;
  const bool rule = a.mode == MODE_IP && !a.raw;
  const int64_t need = rule ? 2 * (int64_t)a.k - 1 : (int64_t)a.k;
  // entries past the rows in place never exist: the last page is never needed
  const int64_t npages = std::max<int64_t>(1, (std::min<int64_t>(need, ntotal) + 63) / 64);
  const int64_t KA = npages * 64;
  const bool gemv_fits =
      (size_t)kGemvMaxQ * idx->ld * sizeof(float) + 4 * kGemvMaxQ * 64 * 8 <= 64 * 1024;
  const bool l2d = a.mode == MODE_L2 && a.l2_direct && idx->esize == 4 && gemv_fits && a.self0 < 0;
  const bool gemv = !gathered && a.self0 < 0 && idx->esize == 4 && gemv_fits &&
                    (l2d || (a.mode == MODE_IP && a.nq <= 2));
  // The staged engine's last stage (gathered, fp32 rows): the pages are the
  // exact-key stream's (vs_exact.hip, floored), every key the rescoring's own
  // (fp64 sums of the exact products, one rounding), so what no filter stage
  // settled is answered strictly like the rest (inner product k > 32, L2 k >
  // 56), not with the fp32 GEMM's keys.  Env VS_EXACT_STREAM=0 keeps the GEMM
  // pages (A/B).
  const bool xpages =
      gathered && idx->esize == 4 && a.self0 < 0 && exact_stream_on() && exact_stream_nq(idx->ld) > 0;
  const int pmode = l2d || (xpages && a.mode == MODE_L2 && a.l2_direct) ? MODE_L2D : a.mode;
  // query windows: GEMV groups of up to 8, else pages of at most ~2 GB
  int64_t W = a.nq;
  if (gemv) {
    W = kGemvMaxQ;
  } else if (!gathered) {
    W = std::max<int64_t>(kBQ, ((int64_t)2 << 30) / (KA * 12) / kBQ * kBQ);
  }
  const int64_t nw_max = std::min<int64_t>(W, a.nq);
  const int64_t nrow = gathered ? a.nq_pad : round_up(std::max<int64_t>(nw_max, kGemvMaxQ), kBQ);
  Scratch scr(st);
  float* Dacc = nullptr;
  int64_t* Iacc = nullptr;
  float* fkey = nullptr;
  int *fid = nullptr, *member = nullptr, *active = nullptr, *qlist = nullptr, *qcount = nullptr;
  VS_HIP(scr.alloc((void**)&Dacc, (size_t)nrow * KA * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&Iacc, (size_t)nrow * KA * sizeof(int64_t)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&fkey, (size_t)nrow * sizeof(float)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&fid, (size_t)nrow * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&member, (size_t)nrow * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&active, (size_t)nrow * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&qlist, (size_t)nrow * sizeof(int)), "vs: scratch");
  VS_HIP(scr.alloc((void**)&qcount, sizeof(int)), "vs: scratch");
  // the page kernels' partial lists
  Partials part;
  part.KP = 64;
  int nsplit = 1, cap = 0, xslots = 0;
  int* wc = nullptr;
  if (gemv) {
    part.P = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (ntotal + 255) / 256));
    VS_HIP(scr.alloc((void**)&part.key, (size_t)kGemvMaxQ * part.P * 64 * sizeof(float)),
           "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, (size_t)kGemvMaxQ * part.P * 64 * sizeof(int)),
           "vs: scratch");
    VS_HIP(scr.alloc((void**)&wc, sizeof(int)), "vs: scratch");
  } else if (xpages) {
    // slots per exact-page launch: the whole gathered batch up to 1,024 (its
    // lists: 1,024 x 256 row blocks x 64 entries = 134 MB), so a page of a
    // 4,096-query search is 4 launch triples, not 16 (they run every search,
    // usually over an empty count)
    part.P = (int)std::min<int64_t>(256, std::max<int64_t>(1, ((int64_t)ntotal + 1023) / 1024));
    xslots = (int)std::min<int64_t>(kXPageSlots, round_up(std::max(a.nq, 1), kBQ));
    VS_HIP(scr.alloc((void**)&part.key, (size_t)xslots * part.P * 64 * sizeof(float)),
           "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, (size_t)xslots * part.P * 64 * sizeof(int)),
           "vs: scratch");
    VS_HIP(scr.alloc((void**)&wc, sizeof(int)), "vs: scratch");
  } else {
    const int ntiles = (ntotal + kBN - 1) / kBN;
    nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(ntiles, 256));
    part.P = 2 * nsplit;
    // gathered slots run in windows whose lists stay within ~1 GB
    cap = (int)std::min<int64_t>(
        nrow, std::max<int64_t>(kBQ, ((int64_t)1 << 30) / ((int64_t)part.P * 64 * 8) / kBQ * kBQ));
    VS_HIP(scr.alloc((void**)&part.key, (size_t)cap * part.P * 64 * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, (size_t)cap * part.P * 64 * sizeof(int)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&wc, sizeof(int)), "vs: scratch");
  }
  for (int64_t q0 = 0; q0 < a.nq; q0 += W) {
    const int nw = (int)std::min<int64_t>(W, a.nq - q0);
    const int nslot = (int)round_up(nw, kBQ);
    // this window's queries (offsets into the staged rows / aux / outputs)
    const int64_t eoff = q0 * idx->ld;
    const float* qf = a.qbuf ? a.qbuf + eoff : nullptr;
    const void* qmat = a.qb16 ? (const void*)((const uint16_t*)a.qb16 + eoff) : (const void*)qf;
    const float* qaux = a.qaux ? a.qaux + q0 : nullptr;
    const int64_t self0 = a.self0 >= 0 ? a.self0 + q0 : -1;
    VS_HIP(hipMemsetAsync(Iacc, 0xFF, (size_t)nw * KA * sizeof(int64_t), st), "vs: pages");
    if (gathered) {
      VS_HIP(hipMemsetAsync(member, 0, (size_t)nw * sizeof(int), st), "vs: pages");
      VS_HIP(hipMemsetAsync(active, 0, (size_t)nw * sizeof(int), st), "vs: pages");
    }
    VS_HIP(launch_page_init(nw, gemv ? kGemvMaxQ : nw, gl, gc, member, active, fkey, fid, st),
           "vs: pages");
    // (exact-key pages: their queries count as the exact stream's, vs_filter_exact_stats)
    unsigned long long* xst = xpages ? device_stats(idx->device) : nullptr;
    VS_HIP(launch_compact_flags(active, nw, qlist, qcount, xst ? xst + 8 : nullptr, nullptr, st),
           "vs: pages");
    for (int64_t p = 0; p < npages; ++p) {
      if (p > 0) {
        VS_HIP(launch_page_step(Dacc, Iacc, KA, (int)p - 1, nw, a.k, rule ? 1 : 0, pmode, active,
                                fkey, fid, st),
               "vs: pages");
        VS_HIP(launch_compact_flags(active, nw, qlist, qcount, nullptr, nullptr, st), "vs: pages");
      }
      if (gemv) {  // every query's lists (finished ones empty); none: the launch exits
        KernelTimer tm(st, p == 0 && !gathered ? "gemv_topk" : nullptr);
        VS_HIP(launch_gemv_topk(64, pmode, nw, idx->codes, idx->esize, qf, idx->ld, ntotal, part.P,
                                part, st, fkey, fid, qcount),
               "vs: gemv_topk launch");
        tm.stop();
        VS_HIP(launch_page_gate(qcount, nw, wc, st), "vs: pages");
        VS_HIP(launch_merge_partials(pmode, part, nw, 64, 0, -INFINITY, Dacc + p * 64,
                                     Iacc + p * 64, KA, st, 1, nullptr, wc),
               "vs: merge launch");
        continue;
      }
      if (xpages) {  // the active queries in launches of xslots (past the count: exit)
        ExactStreamArgs ea;
        ea.X = (const float*)idx->codes;
        ea.xn = idx->norms;
        ea.xinv = a.mode == MODE_COS ? a.xaux : nullptr;
        ea.ld = idx->ld;
        ea.ntotal = ntotal;
        ea.Q = qf;
        ea.qaux = qaux;
        ea.slots = qlist;
        ea.count = qcount;
        ea.nslot = xslots;
        ea.fkey = fkey;
        ea.fid = fid;
        for (int s0 = 0; s0 < nslot; s0 += xslots) {
          ea.s0 = s0;
          VS_HIP(launch_window_count(qcount, s0, xslots, wc, st), "vs: window");
          VS_HIP(launch_exact_stream(64, pmode, ea, part, st), "vs: exact stream");
          VS_HIP(launch_merge_partials(pmode, part, xslots, 64, 0, -INFINITY, Dacc + p * 64,
                                       Iacc + p * 64, KA, st, 1, qlist + s0, wc),
                 "vs: merge launch");
        }
        continue;
      }
      for (int w0 = 0; w0 < nslot; w0 += cap) {
        VS_HIP(launch_window_count(qcount, w0, cap, wc, st), "vs: window");
        KernelTimer tm(st, p == 0 && w0 == 0 && !gathered ? "gemm_topk" : nullptr);
        VS_HIP(launch_gemm_topk(64, a.mode, idx->codes, a.xaux, qmat, qaux, idx->ld, idx->esize,
                                ntotal, cap, nsplit, self0, part, st, qlist + w0, wc, fkey, fid),
               "vs: gemm_topk launch");
        tm.stop();
        VS_HIP(launch_merge_partials(a.mode, part, cap, 64, 0, -INFINITY, Dacc + p * 64,
                                     Iacc + p * 64, KA, st, 1, qlist + w0, wc),
               "vs: merge launch");
      }
    }
    VS_HIP(launch_page_finish(pmode, Dacc, Iacc, KA, nw, a.k, rule ? 1 : 0, member, idx->id_base,
                              a.min_score, a.D + q0 * a.k, a.I + q0 * a.k, st),
           "vs: pages");
  }
  return VS_OK;
}

// Shared search driver: queries already staged in `qbuf` ([nq_pad][ld] device,
// zero-padded) with query aux values (`qaux`, L2 norms or 1/|q|).
int run_topk(vs_index* idx, const SearchArgs& a, hipStream_t st, int force_engine) {
  // faiss's inner-product tie rule (vs_support.hip, faiss_ip_tie_order) needs the
  // lowest 2k-1 (key, label) entries of every partial list to be exact; `raw`
  // output (plain lexicographic order) needs k.
  const int mode = a.mode;
  const bool tie_rule = mode == MODE_IP && !a.raw;
  const int need = tie_rule ? 2 * a.k - 1 : a.k;
  const int ntotal = (int)idx->ntotal;
  const int nq = a.nq;
  int engine = force_engine != VS_ENGINE_AUTO ? force_engine
               : idx->engine != VS_ENGINE_AUTO ? idx->engine
                                               : engine_from_env();
  // Large batches of fp32 indexes: the filter-and-verify engine where it applies
  // (candidates for `need` exact entries: x1_list_len, up to 127 — inner
  // product to k = 64), else (or VS_ENGINE=fp32) the fp32 MFMA GEMM.  bf16
  // indexes: the bf16 MFMA GEMM.
  // (past 64 candidates, inner product only: the last stage for what the
  // filter cannot settle is then the two-page exact engine, inner product's;
  // L2 / cosine with k > 56 keep the exact engine)
  const int KF = x1_list_len(need);
  // the planes this search may run through: int8 first, then bf16; a forced
  // *_VERIFY engine runs its plane alone (an L2 index's int8 plane is the
  // augmented one: L2 searches only)
  bool i8_ok = idx->plane_on[FILTER_I8] && idx->ld + idx->aug_m <= kI8MaxLd &&
               (idx->l2aug() ? mode == MODE_L2 && idx->aug_m > 0 : mode != MODE_L2) &&
               engine != VS_ENGINE_BF16_VERIFY;
  const bool b16_ok = idx->plane_on[FILTER_BF16] && engine != VS_ENGINE_I8_VERIFY &&
                      (idx->l2aug() ? mode == MODE_L2 && idx->aug_m > 0 : true);
  const bool staged = idx->esize == 4 && engine != VS_ENGINE_FP32_MFMA && KF > 0 && ntotal > 0 &&
                      nq > kSkinnyMaxQ && (i8_ok || b16_ok);
  // Small batches over a large index with a filter plane for the metric (inner
  // product; L2 when faiss would take its BLAS branch): the staged engine with
  // skinny passes (below)
  const bool small_staged = small_filter_on() && (idx->esize == 4 || mode == MODE_IP) &&
                            engine == VS_ENGINE_AUTO && KF > 0 && nq <= kSkinnyMaxQ &&
                            a.self0 < 0 && ntotal >= kSmallFilterMinRows &&
                            (mode == MODE_IP || mode == MODE_L2) && (i8_ok || b16_ok) &&
                            small_l2d_ok(mode, a);
  // more entries than one exact page holds (inner product k > 32, raw k > 64)
  // and no filter pass for them: the paged exact engine
  if (need > VS_MAX_K && !staged && !small_staged) return run_paged(idx, a, st);
  const int KP = kp_for(need);

  // Small batches stream the corpus once.  fp32 L2 searches whose CALL has
  // fewer than 20 queries take faiss's sequential branch (direct sum (x-q)^2,
  // faiss's distance_compute_blas_threshold): the GEMV kernel, 8 queries per
  // pass.  Otherwise the skinny MFMA kernel (any metric / dtype, L2 by the norm
  // expansion like faiss's BLAS branch), or the GEMV for one or two inner-product
  // queries on fp32 rows (measured faster there, profiles/r01_small_batch_ab.txt).
  static const char* pref = getenv("VS_SMALL_BATCH");
  const bool small_ok = (mode == MODE_IP || mode == MODE_L2) && a.self0 < 0;
  const bool gemv_fits =
      (size_t)kGemvMaxQ * idx->ld * sizeof(float) + 4 * kGemvMaxQ * 64 * 8 <= 64 * 1024;
  const bool direct = small_ok && mode == MODE_L2 && a.l2_direct && idx->esize == 4 && gemv_fits;
  const bool skinny_ok = small_ok && !direct && nq <= kSkinnyMaxQ && KP <= 32 &&
                         (nq <= 16 || KP <= 16) && (idx->ld * idx->esize) % 64 == 0;
  bool gemv = small_ok && gemv_fits && idx->esize == 4 &&
              (direct || (mode == MODE_IP && nq <= 2 && !(pref && strcmp(pref, "skinny") == 0)));
  if (pref && strcmp(pref, "gemv") == 0 && small_ok && gemv_fits && nq <= kGemvMaxQ &&
      (mode == MODE_IP || direct))
    gemv = true;
  // Small batches over a large fp32 index with a filter plane for the metric
  // (inner product; L2 when faiss would take its BLAS branch): the staged
  // engine with skinny passes — the int8 plane streamed once (a quarter of the
  // fp32 bytes), candidates rescored and proven exactly as for large batches,
  // the few queries it cannot settle through the bf16 plane and the fp32
  // rows (skinny kernels too) — instead of streaming the fp32 rows.
  if (small_staged) {
    if (i8_ok && b16_ok) i8_ok = adaptive_use_i8(idx);
    if (i8_ok) return run_filter_verify(idx, a, need, KF, st, FILTER_I8, !b16_ok);
    return run_filter_verify(idx, a, need, KF, st, FILTER_BF16, false);
  }
  Scratch scr(st);
  Partials part;
  part.KP = KP;
  if (gemv) {
    const int gmode = direct ? MODE_L2D : MODE_IP;
    const int nblocks = (int)std::min<int64_t>(2048, std::max<int64_t>(1, (idx->ntotal + 255) / 256));
    part.P = nblocks;
    const int step = kGemvMaxQ;  // queries per corpus pass
    // the kernel writes lists for its padded query count (1, 2, 4 or 8)
    const int nql = nq <= 2 ? nq : (nq <= 4 ? 4 : kGemvMaxQ);
    const size_t n = (size_t)nql * part.P * KP;
    VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
    for (int q0 = 0; q0 < nq; q0 += step) {
      const int nc = std::min(step, nq - q0);
      KernelTimer tm(st, "gemv_topk");
      VS_HIP(launch_gemv_topk(KP, gmode, nc, idx->codes, idx->esize, a.qbuf + (int64_t)q0 * idx->ld,
                              idx->ld, ntotal, nblocks, part, st),
             "vs: gemv_topk launch");
      tm.stop();
      VS_HIP(launch_merge_partials(gmode, part, nc, a.k, idx->id_base, a.min_score,
                                   a.D + (int64_t)q0 * a.k, a.I + (int64_t)q0 * a.k, a.k, st,
                                   a.raw),
             "vs: merge launch");
    }
    return VS_OK;
  }
  if (skinny_ok) {
    const int nblocks =
        (int)std::min<int64_t>(2048, std::max<int64_t>(1, (idx->ntotal + 255) / 256));
    part.P = nblocks;
    const size_t n = (size_t)nq * part.P * KP;
    VS_HIP(scr.alloc((void**)&part.key, n * sizeof(float)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&part.id, n * sizeof(int)), "vs: scratch");
    const void* qsk = a.qb16 ? a.qb16 : (const void*)a.qbuf;
    KernelTimer tm(st, "skinny_topk");
    VS_HIP(launch_skinny_topk(KP, mode, nq, idx->codes, idx->esize, a.xaux, qsk, a.qaux, idx->ld,
                              ntotal, nblocks, part, st),
           "vs: skinny_topk launch");
    tm.stop();
    VS_HIP(launch_merge_partials(mode, part, nq, a.k, idx->id_base, a.min_score, a.D, a.I, a.k,
                                 st, a.raw),
           "vs: merge launch");
    return VS_OK;
  }
  if (idx->esize == 4 && engine != VS_ENGINE_FP32_MFMA && KF > 0 && ntotal > 0) {
    // the automatic order adapts to how much the int8 stage settles
    if (i8_ok && b16_ok && engine == VS_ENGINE_AUTO) i8_ok = adaptive_use_i8(idx);
    // stages: [int8] -> bf16 with deep lists over what is left -> exact fp32
    if (i8_ok) return run_filter_verify(idx, a, need, KF, st, FILTER_I8, !b16_ok);
    if (b16_ok) return run_filter_verify(idx, a, need, KF, st, FILTER_BF16, false);
  }
  if (need > VS_MAX_K) return run_paged(idx, a, st);
  // No plane serves this metric (the cosine self-join of an L2 index, whose
  // planes hold the rows augmented for L2): the staged engine's last stage over
  // every query — the exact fp32 GEMM, its candidates rescored in fp64 — so the
  // keys are the same exact roundings the planes' searches return.
  const int bp = idx->bstats[FILTER_BF16] ? FILTER_BF16 : idx->bstats[FILTER_I8] ? FILTER_I8 : -1;
  if (idx->esize == 4 && engine != VS_ENGINE_FP32_MFMA && KF > 0 && ntotal > 0 &&
      nq > kSkinnyMaxQ && bp >= 0) {
    int* gl = nullptr;
    int* gc = nullptr;
    VS_HIP(scr.alloc((void**)&gl, (size_t)a.nq_pad * sizeof(int)), "vs: scratch");
    VS_HIP(scr.alloc((void**)&gc, sizeof(int)), "vs: scratch");
    VS_HIP(launch_iota(gl, nq, gc, st), "vs: every query");
    return run_gemm_rescored(idx, a, need, KF, bp, st, gl, gc);
  }
  return run_gemm(idx, a, need, st);
}

}  // namespace

namespace {
int pack_dead(vs_index* idx);
int pack_den();

// Room for n more rows: tombstones are packed first when the rows in place
// would otherwise outgrow the storage, then the storage grows if it must.
int make_room(vs_index* idx, int64_t n, hipStream_t st) {
  if (!idx->dead.empty() && idx->ntotal + n + 256 > idx->capacity) {
    const int rc = pack_dead(idx);
    if (rc) return rc;
  }
  return ensure_capacity(idx, idx->ntotal + n, st);
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
  planes_for(idx);
  idx->ld = round_up(d, 64);  // 64-element K-steps of the filter pass (128-B plane rows)
  *out = idx;
  return VS_OK;
}

int vs_destroy(vs_index* idx) {
  if (!idx) return VS_OK;
  {
    DeviceGuard g(idx->device);
    (void)wait_readers(idx);
    if (idx->wst) (void)hipStreamSynchronize(idx->wst);
    free_storage(idx);
    for (auto& r : idx->readers) (void)hipEventDestroy(r.second);
    idx->readers.clear();
    if (idx->wst) (void)hipStreamDestroy(idx->wst);
    for (int p = 0; p < 2; ++p)
      if (idx->bstats[p]) (void)hipFree(idx->bstats[p]);
    if (idx->ad.dcount) (void)hipFree(idx->ad.dcount);
    if (idx->ddead) (void)hipFree(idx->ddead);
    if (idx->ad.hmirror) (void)hipHostFree(idx->ad.hmirror);
    if (idx->ad.ev) (void)hipEventDestroy(idx->ad.ev);
  }
  delete idx;
  return VS_OK;
}

int vs_reserve(vs_index* idx, int64_t n) {
  if (!idx) return fail(VS_E_INVALID, "vs_reserve: null index");
  if (n < 0) return fail(VS_E_INVALID, "vs_reserve: n < 0");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  // an index that tombstones its removals keeps room for the appends that
  // come before the next pack (1 / pack_den of the rows): at C5's size a
  // storage growth (a copy beside the old rows) does not fit in HBM
  const int64_t want = std::max(n, idx->ntotal);
  if (idx->tombstones() && want / pack_den() > 0) {
    // the headroom is a convenience: without room for it, the exact request
    if (ensure_capacity(idx, want + want / pack_den(), nullptr) == VS_OK) return VS_OK;
    (void)hipGetLastError();
  }
  return ensure_capacity(idx, want, nullptr);
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
  int rc = make_room(idx, n, st);
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
  rc = derive_plane(idx, idx->ntotal, n, st, true);
  if (rc) return rc;
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
  int rc = make_room(idx, n, st);
  if (rc) return rc;
  VS_HIP(launch_fill_synthetic(idx->row(idx->ntotal), idx->esize, n, idx->d, idx->ld, seed, row0,
                               st),
         "vs_add_synthetic: fill");
  VS_HIP(launch_row_norms(idx->codes, idx->esize, idx->ld, idx->ntotal, n, idx->norms, st),
         "vs_add_synthetic: norms");
  rc = derive_plane(idx, idx->ntotal, n, st, true);
  if (rc) return rc;
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
  int rc = make_room(idx, n, st);
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
  rc = derive_plane(idx, idx->ntotal, n, st, true);
  if (rc) return rc;
  VS_HIP(hipStreamSynchronize(st), "vs_add_synthetic_ids: synchronise");
  idx->ntotal += n;
  return VS_OK;
}

int vs_reset(vs_index* idx) {
  if (!idx) return fail(VS_E_INVALID, "vs_reset: null index");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  VS_HIP(wait_readers(idx), "vs_reset");
  free_storage(idx);
  for (int p = 0; p < 2; ++p)
    if (idx->bstats[p]) VS_HIP(hipMemset(idx->bstats[p], 0, 4 * sizeof(unsigned)), "vs_reset");
  idx->ntotal = 0;
  idx->dead.clear();
  // an empty index starts over: the planes a memory shortage dropped come back
  // (the next add allocates them with the rows), and the next add's rows fix a
  // fresh L2 augmentation
  planes_for(idx);
  reset_l2aug(idx);
  return VS_OK;
}

int vs_ntotal(const vs_index* idx, int64_t* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_ntotal: null argument");
  *out = idx->live();  // faiss ntotal: the live rows
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
  if (engine != VS_ENGINE_AUTO && engine != VS_ENGINE_FP32_MFMA &&
      engine != VS_ENGINE_BF16_VERIFY && engine != VS_ENGINE_I8_VERIFY)
    return fail(VS_E_INVALID, "vs_set_engine: unknown engine");
  std::unique_lock<std::shared_mutex> lk(idx->mu);
  if (idx->esize == 4 && engine == VS_ENGINE_I8_VERIFY && !idx->plane_on[FILTER_I8])
    return fail(VS_E_UNSUPPORTED,
                "vs_set_engine: no int8 filter plane (it serves inner-product indexes)");
  if (idx->esize == 4 && engine == VS_ENGINE_BF16_VERIFY && !idx->plane_on[FILTER_BF16])
    return fail(VS_E_UNSUPPORTED, "vs_set_engine: no bf16 filter plane (VS_FILTER=i8)");
  idx->engine = engine;
  return VS_OK;
}

const char* vs_notice(const vs_index* idx) { return idx ? idx->notice.c_str() : ""; }

int vs_filter_plane(const vs_index* idx, int* out) {
  if (!idx || !out) return fail(VS_E_INVALID, "vs_filter_plane: null argument");
  *out = (idx->plane_on[FILTER_I8] ? VS_FILTER_I8 : 0) |
         (idx->plane_on[FILTER_BF16] ? VS_FILTER_BF16 : 0);
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
  // any k, as faiss-cpu's IndexFlat::search (k > 64: the paged exact engine,
  // run_paged); the bound only keeps 2k - 1 inside the engines' int arithmetic
  if (k > INT_MAX / 2) return fail(VS_E_INVALID, "vs_search: k too large");
  if (n == 0) return VS_OK;
  if (!x || !D || !I) return fail(VS_E_INVALID, "vs_search: null buffer");
  hipStream_t st = (hipStream_t)stream;
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  DeviceGuard g(idx->device);
  if (!g.ok) return fail(VS_E_HIP, "vs_search: hipSetDevice failed");
  ReaderMark mark(idx, st);
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
      SearchArgs sa;
      sa.mode = mode;
      sa.qbuf = qbuf;
      sa.qb16 = qb16;
      sa.qaux = qaux;
      sa.xaux = idx->norms;
      sa.nq = (int)nc;
      sa.nq_pad = (int)nq_pad;
      sa.k = (int)k;
      sa.raw = (flags & VS_RAW_ORDER) ? 1 : 0;
      sa.l2_direct = n < kBlasThreshold;  // faiss decides on the whole call's nq
      sa.host_wait = !out_dev;
      sa.D = Dd + c0 * k;
      sa.I = Id + c0 * k;
      int rc = run_topk(idx, sa, st, VS_ENGINE_AUTO);
      if (rc) return rc;
    }
    // tombstoned rows never enter a list; the rows found become faiss labels
    if (!idx->dead.empty())
      VS_HIP(launch_label_map(Id, n * k, idx->ddead, (int64_t)idx->dead.size(), idx->id_base, st),
             "vs_search: labels");
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

}  // extern "C"

namespace {
int reconstruct_rows(vs_index* idx, int64_t i0, int64_t n, float* out, int flags, hipStream_t st);
int64_t row_of_label(const vs_index* idx, int64_t l);
}  // namespace

extern "C" {

int vs_reconstruct_n(vs_index* idx, int64_t i0, int64_t n, float* out, int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_reconstruct_n: null index");
  hipStream_t st = (hipStream_t)stream;
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  if (n < 0 || i0 < 0 || i0 + n > idx->live())
    return fail(VS_E_INVALID, "vs_reconstruct_n: key out of range");  // faiss: FAISS_THROW_IF_NOT
  if (n == 0) return VS_OK;
  if (!out) return fail(VS_E_INVALID, "vs_reconstruct_n: null output");
  DeviceGuard g(idx->device);
  ReaderMark mark(idx, st);
  // labels [i0, i0 + n) are runs of rows in place between tombstones
  int64_t p = row_of_label(idx, i0), done = 0;
  size_t j = std::upper_bound(idx->dead.begin(), idx->dead.end(), p) - idx->dead.begin();
  while (done < n) {
    const int64_t stop = j < idx->dead.size() ? idx->dead[j] : idx->ntotal;
    const int64_t run = std::min(n - done, stop - p);
    const int rc = reconstruct_rows(idx, p, run, out + done * idx->d, flags, st);
    if (rc) return rc;
    done += run;
    p += run;
    while (j < idx->dead.size() && idx->dead[j] == p) ++p, ++j;  // skip the tombstones
  }
  if (!(flags & VS_OUT_DEVICE)) VS_HIP(hipStreamSynchronize(st), "vs_reconstruct_n: synchronise");
  return VS_OK;
}

}  // extern "C"

namespace {
// Rows in place [i0, i0 + n) -> fp32 out (the caller holds the reader lock).
int reconstruct_rows(vs_index* idx, int64_t i0, int64_t n, float* out, int flags, hipStream_t st) {
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
  return VS_OK;
}
}  // namespace

extern "C" {

}  // extern "C"

namespace {
// Stable compaction of the sorted physical rows `rm` out of the index (rows,
// norms, filter planes re-derived over the moved rows), on the writer stream
// `st`, after the index's readers have drained; synchronises.
int compact_rows(vs_index* idx, const std::vector<int64_t>& rm, hipStream_t st) {
  const int64_t nrem = (int64_t)rm.size();
  if (nrem == 0) return VS_OK;
  Scratch scr(st);
  int64_t* drm = nullptr;
  VS_HIP(scr.alloc((void**)&drm, (size_t)nrem * sizeof(int64_t)), "vs_remove_ids: scratch");
  VS_HIP(hipMemcpyAsync(drm, rm.data(), (size_t)nrem * sizeof(int64_t), hipMemcpyHostToDevice, st),
         "vs_remove_ids: upload");
  // Chunked stable compaction from the first removed row on.  A chunk whose
  // rows move down by at least its own length (`before`, the removed rows
  // below it, >= its row count) is packed straight to its final position: its
  // destinations lie below its sources, in rows earlier chunks have already
  // consumed (stream order).  Otherwise (near the first removed row, where the
  // shift is small) the kept rows are packed into scratch, then copied down.
  // Once the shift reaches kDirectMin rows, chunks are cut to the shift so
  // every later chunk takes the direct path (half the bytes moved).
  const int64_t chunk = std::max<int64_t>(1024, (int64_t)(256ull << 20) / idx->rowbytes());
  constexpr int64_t kDirectMin = 16384;
  char* tmp = nullptr;
  float* tmpn = nullptr;
  const int64_t first = rm[0];
  for (int64_t s0 = first, cn = 0; s0 < idx->ntotal; s0 += cn) {
    const int64_t before = std::lower_bound(rm.begin(), rm.end(), s0) - rm.begin();
    cn = std::min(chunk, idx->ntotal - s0);
    const bool direct = before >= cn || before >= kDirectMin;
    if (direct) cn = std::min(cn, before);
    const int64_t in_chunk = std::lower_bound(rm.begin(), rm.end(), s0 + cn) - rm.begin() - before;
    const int64_t kept = cn - in_chunk;
    const int64_t dst = s0 - before;
    if (direct) {
      VS_HIP(launch_gather_kept(idx->codes, idx->norms, idx->rowbytes(), s0, cn, drm + before,
                                in_chunk, idx->row(dst), idx->norms + dst, st),
             "vs_remove_ids: move rows");
      continue;
    }
    if (!tmp) {
      VS_HIP(scr.alloc((void**)&tmp, (size_t)chunk * idx->rowbytes()), "vs_remove_ids: scratch");
      VS_HIP(scr.alloc((void**)&tmpn, (size_t)chunk * sizeof(float)), "vs_remove_ids: scratch");
    }
    VS_HIP(launch_gather_kept(idx->codes, idx->norms, idx->rowbytes(), s0, cn, drm + before,
                              in_chunk, tmp, tmpn, st),
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
  VS_HIP(hipMemsetAsync(idx->row(nt), 0, (size_t)nrem * idx->rowbytes(), st),
         "vs_remove_ids: zero tail");
  VS_HIP(hipMemsetAsync(idx->norms + nt, 0, (size_t)nrem * sizeof(float), st),
         "vs_remove_ids: zero tail");
  // the filter planes are re-derived from the moved rows (one pass over
  // them), and their tails zeroed like the rows'; the bound maxima are
  // recomputed over the remaining rows (a removal can lower them)
  int rc = derive_plane(idx, first, nt - first, st);
  if (rc) return rc;
  for (int p = 0; p < 2; ++p)
    if (idx->plane_on[p] && idx->bstats[p])
      VS_HIP(launch_bound_stats(plane_norms(idx, p), idx->rn2[p], nt, idx->bstats[p], st),
             "vs_remove_ids: bound maxima");
  for (int p = 0; p < 2; ++p) {
    if (!idx->plane_on[p]) continue;
    VS_HIP(launch_plane_zero_rows(idx->fplane[p], idx->planebytes(p), nt, nrem, st),
           "vs_remove_ids: zero tail");
    VS_HIP(hipMemsetAsync(idx->rn2[p] + nt, 0, (size_t)nrem * sizeof(float), st),
           "vs_remove_ids: zero tail");
  }
  if (idx->fscale)
    VS_HIP(hipMemsetAsync(idx->fscale + nt, 0, (size_t)nrem * sizeof(float), st),
           "vs_remove_ids: zero tail");
  if (idx->anorm)
    VS_HIP(hipMemsetAsync(idx->anorm + nt, 0, (size_t)nrem * sizeof(float), st),
           "vs_remove_ids: zero tail");
  if (idx->anorm_b)
    VS_HIP(hipMemsetAsync(idx->anorm_b + nt, 0, (size_t)nrem * sizeof(float), st),
           "vs_remove_ids: zero tail");
  VS_HIP(hipStreamSynchronize(st), "vs_remove_ids: synchronise");
  idx->ntotal = nt;
  return VS_OK;
}

// Tombstoned rows -> packed storage (the same compaction as an immediate
// removal); the labels do not change.
int pack_dead(vs_index* idx) {
  if (idx->dead.empty()) return VS_OK;
  DeviceGuard g(idx->device);
  VS_HIP(wait_readers(idx), "vs: pack");
  hipStream_t st = nullptr;
  VS_HIP(writer_stream(idx, &st), "vs: pack");
  const int rc = compact_rows(idx, idx->dead, st);
  if (rc) return rc;
  idx->dead.clear();
  return VS_OK;
}

// Dead fraction at which a removal packs the tombstones (1 / kPackDen of the
// rows in place; env VS_PACK_DEN overrides, 1 = pack at every removal).  A
// dead row costs every search its bytes until the pack, a pack moves every
// row after the first dead one: at C5's 1 % per mutation round a pack comes
// every ~6 rounds.
int pack_den() {
  const char* e = getenv("VS_PACK_DEN");
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : 16;
}

// Live label l -> its row in place (the sorted dead list skipped).
int64_t row_of_label(const vs_index* idx, int64_t l) {
  int64_t p = l;
  for (int64_t d : idx->dead) {
    if (d <= p) ++p;
    else break;
  }
  return p;
}
}  // namespace

extern "C" {

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
  const int64_t live = idx->live();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t r = ids[i] - idx->id_base;
    if (r >= 0 && r < live) rm.push_back(r);
  }
  std::sort(rm.begin(), rm.end());
  rm.erase(std::unique(rm.begin(), rm.end()), rm.end());
  const int64_t nrem = (int64_t)rm.size();
  if (nrem == 0) return VS_OK;
  DeviceGuard g(idx->device);
  // Searches of this index already queued on other streams read the rows we
  // are about to move or overwrite: wait for their marks (not for the device).
  VS_HIP(wait_readers(idx), "vs_remove_ids: drain");
  hipStream_t st = nullptr;
  VS_HIP(writer_stream(idx, &st), "vs_remove_ids: stream");
  // labels -> rows in place (both ascending: one merge walk over the dead list)
  if (!idx->dead.empty()) {
    size_t j = 0;
    int64_t shift = 0;
    for (auto& r : rm) {
      while (j < idx->dead.size() && idx->dead[j] <= r + shift) ++j, ++shift;
      r += shift;
    }
  }
  if (!idx->tombstones()) {  // filter planes to keep in step: compact now
    const int rc = compact_rows(idx, rm, st);
    if (rc) return rc;
  } else {
    Scratch scr(st);
    int64_t* drm = nullptr;
    VS_HIP(scr.alloc((void**)&drm, (size_t)nrem * sizeof(int64_t)), "vs_remove_ids: scratch");
    VS_HIP(hipMemcpyAsync(drm, rm.data(), (size_t)nrem * sizeof(int64_t), hipMemcpyHostToDevice,
                          st),
           "vs_remove_ids: upload");
    VS_HIP(launch_fill_nan_rows(idx->codes, idx->rowbytes(), idx->norms, idx->esize, drm, nrem, st,
                                idx->plane_on[FILTER_I8] ? idx->fscale : nullptr),
           "vs_remove_ids: tombstones");
    std::vector<int64_t> merged;
    merged.reserve(idx->dead.size() + rm.size());
    std::merge(idx->dead.begin(), idx->dead.end(), rm.begin(), rm.end(),
               std::back_inserter(merged));
    idx->dead.swap(merged);
    VS_HIP(hipStreamSynchronize(st), "vs_remove_ids: synchronise");
    if ((int64_t)idx->dead.size() * pack_den() >= idx->ntotal) {
      const int rc = pack_dead(idx);
      if (rc) return rc;
    } else {
      const int64_t nd = (int64_t)idx->dead.size();
      if (nd > idx->ddead_cap) {
        const int64_t cap = std::max<int64_t>(nd, 2 * idx->ddead_cap);
        if (idx->ddead) (void)hipFree(idx->ddead);
        idx->ddead = nullptr;
        idx->ddead_cap = 0;
        VS_HIP(hipMalloc(&idx->ddead, (size_t)cap * sizeof(int64_t)), "vs_remove_ids: dead list");
        idx->ddead_cap = cap;
      }
      VS_HIP(hipMemcpyAsync(idx->ddead, idx->dead.data(), (size_t)nd * sizeof(int64_t),
                            hipMemcpyHostToDevice, st),
             "vs_remove_ids: dead list");
      VS_HIP(hipStreamSynchronize(st), "vs_remove_ids: synchronise");
    }
  }
  // every row removed: the next add's rows fix a fresh L2 augmentation (the
  // old one followed rows that are gone)
  if (idx->ntotal == 0) reset_l2aug(idx);
  if (nremoved) *nremoved = nrem;
  return VS_OK;
}

int vs_selfjoin(vs_index* idx, int64_t q0, int64_t nq, int64_t k, int exclude_self,
                float min_sim, float* D, int64_t* I, int flags, void* stream) {
  if (!idx) return fail(VS_E_INVALID, "vs_selfjoin: null index");
  if (k <= 0) return fail(VS_E_INVALID, "vs_selfjoin: k must be > 0");
  if (k > INT_MAX / 2) return fail(VS_E_INVALID, "vs_selfjoin: k too large");
  if (q0 < 0 || nq < 0) return fail(VS_E_INVALID, "vs_selfjoin: query rows out of range");
  if (nq > 0 && (!D || !I)) return fail(VS_E_INVALID, "vs_selfjoin: null buffer");
  hipStream_t st = (hipStream_t)stream;
  // The self-join reads its query rows in place and emits row numbers as labels,
  // so it runs on an index without tombstones: under the shared lock it checks
  // for them, and if a removal left some, packs them under the unique lock and
  // looks again (a removal can land between the two locks).
  std::shared_lock<std::shared_mutex> lk(idx->mu);
  while (!idx->dead.empty()) {
    lk.unlock();
    {
      std::unique_lock<std::shared_mutex> wl(idx->mu);
      const int rc = pack_dead(idx);
      if (rc) return rc;
    }
    lk.lock();
  }
  if (q0 + nq > idx->ntotal) return fail(VS_E_INVALID, "vs_selfjoin: query rows out of range");
  if (nq == 0) return VS_OK;
  DeviceGuard g(idx->device);
  ReaderMark mark(idx, st);
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
    SearchArgs sa;
    sa.mode = MODE_COS;
    sa.qbuf = b16 ? nullptr : (const float*)idx->row(qrow);
    sa.qb16 = b16 ? (const void*)idx->row(qrow) : nullptr;
    sa.qaux = rinv + qrow;
    sa.xaux = rinv;
    sa.nq = (int)nc;
    sa.nq_pad = (int)nq_pad;
    sa.k = (int)k;
    sa.self0 = exclude_self ? qrow : -1;
    sa.min_score = min_sim;
    sa.D = Dd + c0 * k;
    sa.I = Id + c0 * k;
    int rc = run_topk(idx, sa, st, VS_ENGINE_AUTO);
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
  if (k > INT_MAX / 2) return fail(VS_E_INVALID, "vs_merge_topk: k too large");
  if (nparts > 64) return fail(VS_E_UNSUPPORTED, "vs_merge_topk: more than 64 parts");
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

// The counters live on the devices (written by the searches' own kernels); reading
// them waits for every search already queued on those devices.
static int read_filter_stats(unsigned long long out[kStatSlots], int reset) {
  for (int i = 0; i < kStatSlots; ++i) out[i] = 0;
  std::lock_guard<std::mutex> g(g_stats_mu);
  for (int dev = 0; dev < (int)g_dev_stats.size(); ++dev) {
    if (!g_dev_stats[dev]) continue;
    DeviceGuard dg(dev);
    unsigned long long h[kStatSlots] = {};
    VS_HIP(hipDeviceSynchronize(), "vs_filter_stats");
    VS_HIP(hipMemcpy(h, g_dev_stats[dev], sizeof(h), hipMemcpyDeviceToHost), "vs_filter_stats");
    for (int i = 0; i < kStatSlots; ++i) out[i] += h[i];
    if (reset) VS_HIP(hipMemset(g_dev_stats[dev], 0, sizeof(h)), "vs_filter_stats");
  }
  return VS_OK;
}

int vs_filter_stats(int64_t* queries, int64_t* fallbacks, int reset) {
  if (!queries || !fallbacks) return fail(VS_E_INVALID, "vs_filter_stats: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, reset);
  if (rc) return rc;
  *queries = (int64_t)c[0];
  *fallbacks = (int64_t)c[2];
  return VS_OK;
}

int vs_filter_wide_stats(int64_t* wide) {
  if (!wide) return fail(VS_E_INVALID, "vs_filter_wide_stats: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, 0);
  if (rc) return rc;
  *wide = (int64_t)c[1];
  return VS_OK;
}

int vs_filter_wide_sets(int64_t* entries, int64_t* rescored) {
  if (!entries || !rescored) return fail(VS_E_INVALID, "vs_filter_wide_sets: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, 0);
  if (rc) return rc;
  *entries = (int64_t)c[4];
  *rescored = (int64_t)c[5];
  return VS_OK;
}

int vs_filter_dump_stats(int64_t* dumps, int64_t* overflows) {
  if (!dumps || !overflows) return fail(VS_E_INVALID, "vs_filter_dump_stats: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, 0);
  if (rc) return rc;
  *dumps = (int64_t)c[6];
  *overflows = (int64_t)c[7];
  return VS_OK;
}

int vs_filter_second_stats(int64_t* second) {
  if (!second) return fail(VS_E_INVALID, "vs_filter_second_stats: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, 0);
  if (rc) return rc;
  *second = (int64_t)c[3];
  return VS_OK;
}

int vs_filter_exact_stats(int64_t* streamed) {
  if (!streamed) return fail(VS_E_INVALID, "vs_filter_exact_stats: null output");
  unsigned long long c[kStatSlots];
  int rc = read_filter_stats(c, 0);
  if (rc) return rc;
  *streamed = (int64_t)c[8];
  return VS_OK;
}

int vs_x1_stamps(unsigned long long* out, int reset) {
  if (!out) return fail(VS_E_INVALID, "vs_x1_stamps: null buffer");
  VS_HIP(x1_stamps(out, reset), "vs_x1_stamps");
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
  return vs_timer_read_kernel(nullptr, total_ms, launches);
}

int vs_timer_read_kernel_share(const char* kernel, double* total_ms, int64_t* launches,
                               double* share) {
  if (!total_ms || !launches) return fail(VS_E_INVALID, "vs_timer_read: null output");
  std::lock_guard<std::mutex> g(g_timer_mu);
  double tot = 0.0, sh = 0.0;
  int64_t n = 0;
  for (auto& p : g_timer_events) {
    if (kernel ? strcmp(kernel, p.name) != 0 : p.aux) continue;
    VS_HIP(hipEventSynchronize(p.b), "vs_timer_read: synchronise");
    float ms = 0.0f;
    VS_HIP(hipEventElapsedTime(&ms, p.a, p.b), "vs_timer_read: elapsed");
    tot += ms;
    n += p.dispatches;
    sh += p.share;
  }
  *total_ms = tot;
  *launches = n;
  if (share) *share = sh;
  return VS_OK;
}

int vs_timer_read_kernel(const char* kernel, double* total_ms, int64_t* launches) {
  return vs_timer_read_kernel_share(kernel, total_ms, launches, nullptr);
}

}  // extern "C"
