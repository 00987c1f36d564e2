/*
 * ORACLE — test / baseline infrastructure only (see oracle/flat.py header for
 * the rules).  NOT a parity oracle: timing stand-in for faiss's SPEED.
 *
 * faiss-cpu 1.11.0 runs the nq = 1 search of the reference's live shape
 * (mcp_book_server.py:142 -> IndexFlat::search, sequential branch) on one
 * thread with fvec_inner_product / fvec_L2sqr from faiss/utils/distances_simd.cpp,
 * whose loops are compiled with FAISS_PRAGMA_IMPRECISE_LOOP: the compiler may
 * reassociate the sum, so AVX2 builds keep 8-lane partial sums (two or more
 * registers interleaved) and add them at the end.  oracle_knn_seq
 * (faiss_flat.c) keeps the strict scalar order the parity tests need and runs
 * slower than that (one dependent add chain per row, against a scan that one
 * thread runs at its memory bandwidth); this file restates the reassociated
 * form (16 partial sums = two 8-lane AVX2 registers, fused multiply-adds, one
 * horizontal add)
 * with the same heap (faiss_flat.c's heap discipline, restated below), so
 * bench.py's cpu_baseline.batch1 can report the faiss-speed figure beside the
 * scalar one.  Scores may differ from the scalar order in the last bits; the
 * labels of well-separated top-k lists do not.
 *
 * Built -O3 -mavx2 -mfma (oracle/Makefile): AVX2 + FMA is present on every
 * x86-64 host this runs on (the GPU box's EPYC and this container's Xeon).
 */
#include <float.h>
#include <immintrin.h>
#include <stdint.h>
#include <string.h>

typedef int64_t idx_t;

static inline int cmp2(int is_max, float a1, float b1, idx_t a2, idx_t b2) {
  return is_max ? ((a1 > b1) || ((a1 == b1) && (a2 > b2)))
                : ((a1 < b1) || ((a1 == b1) && (a2 < b2)));
}

/* faiss/utils/Heap.h heap_replace_top (1-based) */
static void replace_top(int is_max, size_t k, float* v, idx_t* ids, float val, idx_t id) {
  v--;
  ids--;
  size_t i = 1;
  for (;;) {
    size_t i1 = i << 1, i2 = i1 + 1, c;
    if (i1 > k) break;
    c = (i2 == k + 1 || cmp2(is_max, v[i1], v[i2], ids[i1], ids[i2])) ? i1 : i2;
    if (cmp2(is_max, val, v[c], id, ids[c])) break;
    v[i] = v[c];
    ids[i] = ids[c];
    i = c;
  }
  v[i] = val;
  ids[i] = id;
}

static inline float hsum8(__m256 a) {
  __m128 s = _mm_add_ps(_mm256_castps256_ps128(a), _mm256_extractf128_ps(a, 1));
  s = _mm_add_ps(s, _mm_movehl_ps(s, s));
  s = _mm_add_ss(s, _mm_shuffle_ps(s, s, 1));
  return _mm_cvtss_f32(s);
}

static inline float ip16(const float* x, const float* y, size_t d) {
  __m256 a0 = _mm256_setzero_ps(), a1 = _mm256_setzero_ps();
  size_t i = 0;
  for (; i + 16 <= d; i += 16) {
    a0 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i), a0);
    a1 = _mm256_fmadd_ps(_mm256_loadu_ps(x + i + 8), _mm256_loadu_ps(y + i + 8), a1);
  }
  float s = hsum8(_mm256_add_ps(a0, a1));
  for (; i < d; i++) s += x[i] * y[i];
  return s;
}

static inline float l2_16(const float* x, const float* y, size_t d) {
  __m256 a0 = _mm256_setzero_ps(), a1 = _mm256_setzero_ps();
  size_t i = 0;
  for (; i + 16 <= d; i += 16) {
    const __m256 t0 = _mm256_sub_ps(_mm256_loadu_ps(x + i), _mm256_loadu_ps(y + i));
    const __m256 t1 = _mm256_sub_ps(_mm256_loadu_ps(x + i + 8), _mm256_loadu_ps(y + i + 8));
    a0 = _mm256_fmadd_ps(t0, t0, a0);
    a1 = _mm256_fmadd_ps(t1, t1, a1);
  }
  float s = hsum8(_mm256_add_ps(a0, a1));
  for (; i < d; i++) {
    const float t = x[i] - y[i];
    s += t * t;
  }
  return s;
}

/* One thread per query (faiss parallelises the sequential branch over
 * queries only; nq = 1 is one thread).  Output: the k best, best first. */
void oracle_knn_seq_simd(const float* x, const float* y, int64_t d, int64_t nq, int64_t ny,
                         int64_t k, int metric, float* D, idx_t* I) {
  const int is_max = metric == 1;
  for (int64_t q = 0; q < nq; q++) {
    const float* xq = x + q * d;
    float* hv = D + q * k;
    idx_t* hi = I + q * k;
    for (int64_t j = 0; j < k; j++) {
      hv[j] = is_max ? FLT_MAX : -FLT_MAX;
      hi[j] = -1;
    }
    for (int64_t j = 0; j < ny; j++) {
      const float dis = is_max ? l2_16(xq, y + j * d, (size_t)d) : ip16(xq, y + j * d, (size_t)d);
      if (is_max ? hv[0] > dis : hv[0] < dis) replace_top(is_max, (size_t)k, hv, hi, dis, j);
    }
    /* best first (insertion sort of the k entries; heap_reorder's order) */
    for (int64_t a = 1; a < k; a++) {
      const float v = hv[a];
      const idx_t id = hi[a];
      int64_t b = a;
      for (; b > 0 && cmp2(is_max, hv[b - 1], v, hi[b - 1], id); b--) {
        hv[b] = hv[b - 1];
        hi[b] = hi[b - 1];
      }
      hv[b] = v;
      hi[b] = id;
    }
  }
}
