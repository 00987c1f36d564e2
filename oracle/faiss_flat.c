/*
 * ORACLE — test infrastructure only (see oracle/flat.py header for the rules).
 *
 * C restatement of faiss-cpu 1.11.0 IndexFlat::search, sequential branch
 * (faiss/utils/distances.cpp exhaustive_L2sqr_seq / exhaustive_inner_product_seq
 * with HeapBlockResultHandler; faiss/utils/Heap.h heap_replace_top / heap_pop /
 * heap_reorder; faiss/utils/ordered_key_value.h CMax / CMin).  faiss is not
 * vendored in /root/reference (pinned at poetry.lock:866-867); this file follows
 * the published algorithm statement by statement so that tie behaviour is the
 * heap's, not an approximation of it:
 *
 *   L2  : CMax heap on dis = sum (x-y)^2 ; cmp(a,b) = a > b ;
 *         cmp2(a1,b1,i1,i2) = a1 > b1 || (a1 == b1 && i1 > i2)
 *   IP  : CMin heap on dis = sum x*y     ; cmp(a,b) = a < b ;
 *         cmp2(a1,b1,i1,i2) = a1 < b1 || (a1 == b1 && i1 < i2)
 *   scan j = 0..n-1 :  if (C::cmp(heap_dis[0], dis)) heap_replace_top(k, dis, j)
 *   k == 1 (Top1 handler): if (C::cmp(best, dis)) best = dis, idx = j
 *   output: heap_reorder (k entries; missing ones are (neutral, -1))
 *   neutral: CMax -> FLT_MAX, CMin -> -FLT_MAX (numeric_limits max / lowest)
 *
 * Build: make -C oracle  (-> oracle/build/liboracle_faiss.so, OpenMP over queries,
 * as faiss parallelises the sequential branch over queries only).
 */
#include <float.h>
#include <stdint.h>
#include <string.h>

typedef int64_t idx_t;

static inline int cmp_max(float a, float b) { return a > b; }
static inline int cmp2_max(float a1, float b1, idx_t a2, idx_t b2) {
  return (a1 > b1) || ((a1 == b1) && (a2 > b2));
}
static inline int cmp_min(float a, float b) { return a < b; }
static inline int cmp2_min(float a1, float b1, idx_t a2, idx_t b2) {
  return (a1 < b1) || ((a1 == b1) && (a2 < b2));
}

/* heap_replace_top<C> (1-based indexing, as in faiss/utils/Heap.h) */
static void heap_replace_top(int is_max, size_t k, float* bh_val, idx_t* bh_ids, float val,
                             idx_t id) {
  bh_val--;
  bh_ids--;
  size_t i = 1, i1, i2;
  for (;;) {
    i1 = i << 1;
    i2 = i1 + 1;
    if (i1 > k) break;
    int c12 = is_max ? cmp2_max(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2])
                     : cmp2_min(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2]);
    if ((i2 == k + 1) || c12) {
      int stop = is_max ? cmp2_max(val, bh_val[i1], id, bh_ids[i1])
                        : cmp2_min(val, bh_val[i1], id, bh_ids[i1]);
      if (stop) break;
      bh_val[i] = bh_val[i1];
      bh_ids[i] = bh_ids[i1];
      i = i1;
    } else {
      int stop = is_max ? cmp2_max(val, bh_val[i2], id, bh_ids[i2])
                        : cmp2_min(val, bh_val[i2], id, bh_ids[i2]);
      if (stop) break;
      bh_val[i] = bh_val[i2];
      bh_ids[i] = bh_ids[i2];
      i = i2;
    }
  }
  bh_val[i] = val;
  bh_ids[i] = id;
}

/* heap_pop<C>: remove the top, last element sifts down (faiss/utils/Heap.h) */
static void heap_pop(int is_max, size_t k, float* bh_val, idx_t* bh_ids) {
  bh_val--;
  bh_ids--;
  float val = bh_val[k];
  idx_t id = bh_ids[k];
  size_t i = 1, i1, i2;
  for (;;) {
    i1 = i << 1;
    i2 = i1 + 1;
    if (i1 > k) break;
    int c12 = is_max ? cmp2_max(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2])
                     : cmp2_min(bh_val[i1], bh_val[i2], bh_ids[i1], bh_ids[i2]);
    if ((i2 == k + 1) || c12) {
      int stop = is_max ? cmp2_max(val, bh_val[i1], id, bh_ids[i1])
                        : cmp2_min(val, bh_val[i1], id, bh_ids[i1]);
      if (stop) break;
      bh_val[i] = bh_val[i1];
      bh_ids[i] = bh_ids[i1];
      i = i1;
    } else {
      int stop = is_max ? cmp2_max(val, bh_val[i2], id, bh_ids[i2])
                        : cmp2_min(val, bh_val[i2], id, bh_ids[i2]);
      if (stop) break;
      bh_val[i] = bh_val[i2];
      bh_ids[i] = bh_ids[i2];
      i = i2;
    }
  }
  bh_val[i] = bh_val[k];
  bh_ids[i] = bh_ids[k];
}

/* heap_reorder<C>: sorted output, missing entries (neutral, -1) at the end */
static void heap_reorder(int is_max, size_t k, float* bh_val, idx_t* bh_ids) {
  size_t i, ii;
  for (i = 0, ii = 0; i < k; i++) {
    float val = bh_val[0];
    idx_t id = bh_ids[0];
    heap_pop(is_max, k - i, bh_val, bh_ids);
    bh_val[k - ii - 1] = val;
    bh_ids[k - ii - 1] = id;
    if (id != -1) ii++;
  }
  memmove(bh_val, bh_val + k - ii, ii * sizeof(*bh_val));
  memmove(bh_ids, bh_ids + k - ii, ii * sizeof(*bh_ids));
  for (; ii < k; ii++) {
    bh_val[ii] = is_max ? FLT_MAX : -FLT_MAX;
    bh_ids[ii] = -1;
  }
}

/* fvec_L2sqr / fvec_inner_product (scalar reference order) */
static inline float l2sqr(const float* x, const float* y, size_t d) {
  float s = 0.0f;
  for (size_t i = 0; i < d; i++) {
    const float t = x[i] - y[i];
    s += t * t;
  }
  return s;
}

static inline float inner(const float* x, const float* y, size_t d) {
  float s = 0.0f;
  for (size_t i = 0; i < d; i++) s += x[i] * y[i];
  return s;
}

/*
 * knn_seq: metric 1 = L2 (CMax), 0 = IP (CMin).
 * x: nq x d queries, y: ny x d database, D/I: nq x k outputs.
 * valid (optional, nq x ny bytes): rows with 0 are skipped (self-exclusion tests).
 */
void oracle_knn_seq(const float* x, const float* y, int64_t d, int64_t nq, int64_t ny,
                    int64_t k, int metric, const uint8_t* valid, float* D, idx_t* I) {
  const int is_max = metric == 1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t q = 0; q < nq; q++) {
    const float* xq = x + q * d;
    float* hv = D + q * k;
    idx_t* hi = I + q * k;
    if (k == 1) {
      float best = is_max ? FLT_MAX : -FLT_MAX;
      idx_t bi = -1;
      for (int64_t j = 0; j < ny; j++) {
        if (valid && !valid[q * ny + j]) continue;
        const float dis = is_max ? l2sqr(xq, y + j * d, (size_t)d) : inner(xq, y + j * d, (size_t)d);
        if (is_max ? cmp_max(best, dis) : cmp_min(best, dis)) {
          best = dis;
          bi = j;
        }
      }
      hv[0] = best;
      hi[0] = bi;
      continue;
    }
    for (int64_t j = 0; j < k; j++) {
      hv[j] = is_max ? FLT_MAX : -FLT_MAX;
      hi[j] = -1;
    }
    for (int64_t j = 0; j < ny; j++) {
      if (valid && !valid[q * ny + j]) continue;
      const float dis = is_max ? l2sqr(xq, y + j * d, (size_t)d) : inner(xq, y + j * d, (size_t)d);
      if (is_max ? cmp_max(hv[0], dis) : cmp_min(hv[0], dis))
        heap_replace_top(is_max, (size_t)k, hv, hi, dis, j);
    }
    heap_reorder(is_max, (size_t)k, hv, hi);
  }
}

/* Same heap discipline over precomputed scores (used to pin the numpy tie rule). */
void oracle_heap_select(const float* scores, int64_t nq, int64_t ny, int64_t k, int metric,
                        float* D, idx_t* I) {
  const int is_max = metric == 1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t q = 0; q < nq; q++) {
    const float* s = scores + q * ny;
    float* hv = D + q * k;
    idx_t* hi = I + q * k;
    for (int64_t j = 0; j < k; j++) {
      hv[j] = is_max ? FLT_MAX : -FLT_MAX;
      hi[j] = -1;
    }
    for (int64_t j = 0; j < ny; j++) {
      if (is_max ? cmp_max(hv[0], s[j]) : cmp_min(hv[0], s[j]))
        heap_replace_top(is_max, (size_t)k, hv, hi, s[j], j);
    }
    heap_reorder(is_max, (size_t)k, hv, hi);
  }
}
