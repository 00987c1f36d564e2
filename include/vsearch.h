/*
 * vsearch.h — C-ABI of libvsearch.so, the MI355X-native exact flat-index engine.
 *
 * This is the drop-in boundary for the reference's one data-parallel hot path:
 * brute-force top-k over 1536-d book / student embeddings.  In the reference the
 * path is reached through LangChain's `FAISS` vector store
 * (langchain-community 0.3.26, /root/reference/poetry.lock:1577-1578) whose
 * `.index` is a faiss-cpu 1.11.0 `IndexFlatL2` / `IndexFlatIP`
 * (/root/reference/poetry.lock:866-867), plus the pgvector cosine top-15
 * self-join in /root/reference/src/graph_refresher/main.py:339-354.
 *
 * Every entry point below names the reference interface it replaces.  faiss and
 * langchain are not vendored in /root/reference; their call sites are cited.
 *
 * Conventions
 *   - every function returns 0 on success, a negative VS_E* code on failure;
 *     the message is available from vs_last_error() (thread-local).
 *   - vectors are C-contiguous float32 rows of length d (what faiss's SWIG layer
 *     receives after np.ascontiguousarray(x, dtype="float32")).
 *   - `flags` say where caller buffers live (VS_IN_DEVICE / VS_OUT_DEVICE);
 *     device buffers must be on the index's device.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).  Calls with
 *     host outputs synchronise that stream before returning.
 *   - labels are int64, exactly faiss's idx_t; padding label is -1.
 */
#ifndef VSEARCH_H
#define VSEARCH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Metric codes equal faiss::MetricType so index.metric_type passes straight through. */
#define VS_METRIC_INNER_PRODUCT 0
#define VS_METRIC_L2 1

/* Storage dtype of the database rows. */
#define VS_DTYPE_F32 0
#define VS_DTYPE_BF16 1

/* Buffer-location flags. */
#define VS_IN_DEVICE 1  /* input vectors / ids are device pointers */
#define VS_OUT_DEVICE 2 /* output buffers are device pointers      */
/* vs_search: return the k entries with the lexicographically smallest
 * (key, label), key = distance (L2) or -score (IP), in that order, instead of
 * faiss's inner-product tie order.  The per-shard half of an exact row-sharded
 * search: faiss's IP tie rule is a function of the 2k-1 best (key, label) pairs
 * of the union, so each shard returns its raw best 2k-1 (any k) and
 * vs_merge_topk applies the rule once (vsearch/sharded.py).  No effect on L2. */
#define VS_RAW_ORDER 4

/* Status codes. */
#define VS_OK 0
#define VS_E_INVALID (-1) /* bad argument (faiss: FAISS_THROW_IF_NOT / assert) */
#define VS_E_HIP (-2)     /* HIP runtime / launch error                        */
#define VS_E_OOM (-3)     /* device allocation failed                          */
#define VS_E_UNSUPPORTED (-4)

/* The entries one exact page holds (register lists of 64).  Not a limit on k:
 * searches and self-joins that need more — k > 64, raw k > 64, faiss's
 * inner-product tie rule at k > 32 — read further pages of 64, each after the
 * previous page's last (key, label) (vs_api.hip run_paged), as faiss-cpu's
 * IndexFlat::search answers any k. */
#define VS_MAX_K 64

typedef struct vs_index vs_index;

/* Thread-local text of the last error (faiss: FaissException::what()). */
const char* vs_last_error(void);
/* Library ABI version (major*10000 + minor*100 + patch). */
int vs_version(void);
/* Number of visible HIP devices. */
int vs_device_count(int* n);

/* ---- index lifetime -------------------------------------------------------
 * Replaces faiss.IndexFlatL2(d) / faiss.IndexFlatIP(d), created by
 * FAISS.from_texts (default EUCLIDEAN => IndexFlatL2) at
 * src/ingestion_service/pipeline.py:359, src/incremental_workers/book_vector/main.py:121,469,
 * src/recommendation_api/candidate_builder.py:69-71, src/recommendation_api/service.py:370-372. */
int vs_create(int d, int metric, int dtype, int device, vs_index** out);
int vs_destroy(vs_index* idx);

/* Pre-size device storage for n rows (no faiss equivalent; avoids regrowth copies). */
int vs_reserve(vs_index* idx, int64_t n);

/* faiss Index::add(n, x) — appends rows; labels continue at ntotal.
 * Callers: FAISS.add_texts at src/ingestion_service/pipeline.py:363,
 * src/incremental_workers/book_vector/main.py:148. */
int vs_add(vs_index* idx, const float* x, int64_t n, int flags, void* stream);

/* Appends n rows of the deterministic counter-based synthetic corpus
 * (row r = global row row0 + i; see vs_fill_synthetic).  Benchmark/test feed only. */
int vs_add_synthetic(vs_index* idx, int64_t n, uint64_t seed, int64_t row0, void* stream);

/* Appends n rows whose synthetic generator row numbers are ids[0..n) (host int64
 * array): row j of the append equals row ids[j] of vs_fill_synthetic's corpus.
 * Lets a benchmark rebuild any mutated corpus exactly.  Benchmark/test feed only. */
int vs_add_synthetic_ids(vs_index* idx, const int64_t* ids, int64_t n, uint64_t seed,
                         void* stream);

/* faiss Index::reset(). */
int vs_reset(vs_index* idx);

/* faiss Index::ntotal / ::d / ::metric_type (read at book_vector/main.py:162-170,
 * ingestion_service/pipeline.py:186,524). */
int vs_ntotal(const vs_index* idx, int64_t* out);
int vs_dim(const vs_index* idx, int* out);
int vs_metric(const vs_index* idx, int* out);
int vs_dtype(const vs_index* idx, int* out);

/* Arithmetic engine of the large-batch path of fp32 indexes:
 *   VS_ENGINE_AUTO          library default where it applies (IP k <= 28, L2 /
 *                           cosine k <= 56), else FP32_MFMA: filter and verify
 *                           in stages over the index's filter planes — int8
 *                           (inner product and cosine), then bf16 for the
 *                           queries the int8 bound cannot settle, then the exact
 *                           FP32_MFMA for what remains;
 *                           env VS_ENGINE=fp32|bf16v|i8v overrides
 *   VS_ENGINE_FP32_MFMA     v_mfma_f32_32x32x2_f32 on the fp32 rows
 *   VS_ENGINE_I8_VERIFY     filter and verify on the int8 plane alone: one int8
 *                           MFMA product per fp32 product (int8 codes of rows
 *                           and queries, one scale per row) keeps the best
 *                           candidates of every query, a rigorous error bound
 *                           proves the exact top-k is among them, the candidates
 *                           are rescored exactly, and queries the bound cannot
 *                           settle are redone by FP32_MFMA — results identical to
 *                           an exact engine
 *   VS_ENGINE_BF16_VERIFY   the same on the bf16 (round-to-nearest-even) plane
 * New fp32 indexes hold the int8 plane (inner product) and the bf16 plane;
 * env VS_FILTER=bf16|i8 at creation keeps one.  bf16 indexes ignore the
 * setting (bf16 MFMA on the stored values). */
#define VS_ENGINE_AUTO 0
#define VS_ENGINE_FP32_MFMA 1
#define VS_ENGINE_BF16_VERIFY 3
#define VS_ENGINE_I8_VERIFY 4
int vs_set_engine(vs_index* idx, int engine);

/* The filter planes an fp32 index holds, a bit set: VS_FILTER_I8 (int8 codes +
 * per-row scale; inner-product indexes) | VS_FILTER_BF16; 0 for bf16 indexes.
 * Library-specific (faiss has no counterpart); the benchmark reads it to price
 * the filter pass. */
#define VS_FILTER_I8 1
#define VS_FILTER_BF16 2
int vs_filter_plane(const vs_index* idx, int* out);
/* The last notice of the index: a filter plane dropped because HBM ran short
 * while the storage grew (searches stay exact on the plane that remains or the
 * exact fp32 engine, but slower); "" if none.  Library-specific.  The pointer
 * stays valid until the next mutation of the index. */
const char* vs_notice(const vs_index* idx);

/* Rows [0,ntotal) get labels id_base + row.  Used by the row-sharded multi-GPU
 * index so that per-shard results carry global faiss labels. */
int vs_set_id_base(vs_index* idx, int64_t id_base);

/* faiss IndexFlat::search(n, x, k, D, I) (knn_L2sqr / knn_inner_product):
 * exact top-k, D ascending squared-L2 or descending inner product, k > ntotal
 * padded with (+FLT_MAX | -FLT_MAX, -1).  Ties follow faiss's heaps: L2 keeps the
 * lower label first; inner product follows faiss's CMin-heap rule (equal scores
 * come out in DESCENDING label order, and which tied labels stay depends on the
 * labels of the better rows — vs_support.hip faiss_ip_tie_order, exact for
 * every k: the rule reads up to the 2k-1 best entries, taken from further
 * pages where the k-th key's run of equal keys fills a page).  Any k > 0
 * (k > ntotal pads; k > INT_MAX/2: VS_E_INVALID).  L2 calls with n < 20 use faiss's sequential branch (direct sum of
 * squares), n >= 20 the BLAS branch (|q|^2 + |x|^2 - 2 q.x clamped at 0).
 * Stream-ordered on `stream` when every buffer is on the device; the call
 * returns once its first filter stage's count of unsettled queries is known
 * (a 4-byte read; later stages are enqueued only for queries left; env
 * VS_TAIL_WAIT=0 or a capturing stream: fully asynchronous, every launch kept).
 * Caller: FAISS.similarity_search_with_score_by_vector, reached from
 * src/recommendation_api/mcp_book_server.py:142, candidate_builder.py:187,321,
 * service.py:529,627.  D is n*k float32, I is n*k int64. */
int vs_search(vs_index* idx, const float* x, int64_t n, int64_t k, float* D, int64_t* I,
              int flags, void* stream);

/* faiss Index::reconstruct_n(i0, n, out) / reconstruct(i) — rows as added
 * (bf16 storage returns the stored bf16 value widened to float32).
 * Callers: store.index.reconstruct at candidate_builder.py:166-168, service.py:490-494. */
int vs_reconstruct_n(vs_index* idx, int64_t i0, int64_t n, float* out, int flags, void* stream);

/* faiss IndexFlat::remove_ids(IDSelectorBatch(ids)) — stable compaction; ids
 * outside [0,ntotal) and duplicates are ignored; *nremoved = rows removed.
 * Caller: langchain FAISS.delete (BASELINE config 5 add/remove). */
int vs_remove_ids(vs_index* idx, const int64_t* ids, int64_t n, int64_t* nremoved);

/* Cosine self-join — replaces the per-student pgvector query
 *   SELECT student_id, 1-(vec <=> src.vec) ... WHERE student_id <> $1
 *   ORDER BY vec <=> src.vec LIMIT 15
 * at src/graph_refresher/main.py:339-354 and src/incremental_workers/similarity/main.py:80-87.
 * For stored rows q in [q0, q0+nq): the k rows with largest cosine similarity
 * dot/sqrt(|a|^2 |b|^2) (ties: lower row first; any k, as SQL's LIMIT), excluding row q itself when
 * exclude_self != 0.  Entries whose similarity is < min_sim (the
 * graph_refresher's S.similarity_threshold filter, main.py:350-354) are returned
 * as (-FLT_MAX, -1).  Zero-norm rows never match (pgvector yields NaN for them).
 * D is nq*k similarities, I is nq*k labels (id_base applied). */
int vs_selfjoin(vs_index* idx, int64_t q0, int64_t nq, int64_t k, int exclude_self,
                float min_sim, float* D, int64_t* I, int flags, void* stream);

/* Merge nparts per-shard top-k lists into one (faiss: the ResultHandler merge;
 * GPU-side half of the RCCL all-gather top-k merge).  Inputs are DEVICE arrays
 * laid out [nparts][nq][k_in] (scores + int64 labels, -1 = empty; raw order for
 * inner product, any k_in and k, nparts <= 64); outputs are DEVICE arrays
 * [nq][k].  metric picks the order (L2 ascending, IP descending). */
int vs_merge_topk(const float* D_parts, const int64_t* I_parts, int64_t nparts, int64_t nq,
                  int64_t k_in, int64_t k, int metric, float* D, int64_t* I, void* stream);

/* Writes rows x[i][j] = ((splitmix64(seed ^ ((row0+i)*d + j)) >> 40) * 2^-23) - 1
 * (exactly representable float32 in [-1,1)) into a DEVICE buffer of rows*d floats.
 * The same generator is restated in python for the oracle (vsearch.synth). */
int vs_fill_synthetic(float* out, int64_t rows, int64_t d, uint64_t seed, int64_t row0,
                      void* stream);

/* ---- measurement ----------------------------------------------------------
 * When enabled, every launch of the dominant search kernel (the fused
 * distance+top-k kernel) is bracketed by HIP events on the launch stream.
 * vs_timer_read synchronises those events and returns the summed kernel time in
 * milliseconds and the number of kernel dispatches inside the timed spans since
 * the last reset (gemm_topk_x1 cuts one search into several dispatches). */
int vs_timer_enable(int on);
/* Queries searched by the filter-and-verify engine and how many of them the
 * exact engine had to redo, since the last reset (reset != 0 clears them). */
int vs_filter_stats(int64_t* queries, int64_t* fallbacks, int reset);
/* Of those queries, how many the first check flagged and the wide check (every
 * lane-list entry below the list floors rescored) examined again, since the last
 * vs_filter_stats reset.  Diagnostic only: no reference interface. */
int vs_filter_wide_stats(int64_t* wide);
/* Queries the staged engine handed from the int8 plane to the bf16 plane since
 * the last vs_filter_stats reset.  Diagnostic only: no reference interface. */
int vs_filter_second_stats(int64_t* second);
/* Queries the staged engine's last stage could not prove from its fp32 GEMM
 * candidates (dense near-ties inside the fp32 bound) and ranked over every row
 * by the exact key instead (vs_exact.hip), since the last vs_filter_stats
 * reset.  Diagnostic only: no reference interface. */
int vs_filter_exact_stats(int64_t* streamed);
/* Entries the wide checks examined (summed over queries) and how many of them
 * were read from HBM and rescored (the rest reuse the first check's exact keys),
 * since the last vs_filter_stats reset.  Diagnostic only: no reference interface. */
int vs_filter_wide_sets(int64_t* entries, int64_t* rescored);
/* Rows the filter pass's dump launches stored (one (row, raw sum) slot per
 * row that may lie below its lane list's floor) and lane lists that ran out of
 * dump slots
 * (their queries went to the next stage), since the last vs_filter_stats
 * reset.  Diagnostic only: no reference interface. */
int vs_filter_dump_stats(int64_t* dumps, int64_t* overflows);
int vs_timer_reset(void);
/* Diagnostic only (no reference interface): the filter pass's per-segment
 * cycle sums of a stamp build (VS_X1_STAMP=1; zeros otherwise), 26 values:
 * [waves 0-3 | 4-7][load issue, vmcnt wait, barrier 1, matrix issue,
 * barrier 2, epilogue, epilogue reject, factor loads, keys and inserts;
 * factor-load paths, inserting blocks, inserts]
 * then the steps of each group; reset != 0 clears them. */
int vs_x1_stamps(unsigned long long* out, int reset);
int vs_timer_read(double* total_ms, int64_t* launches);
/* The same for the spans of one kernel name only (the filter engine's first
 * stage is "gemm_topk_x1_i8" or "gemm_topk_x1" (bf16) per search; its first
 * launch, when the later ones dump, "<name>_list"; the whole pass including
 * the cut and replay kernels "<name>_pass", a span that vs_timer_read's total
 * leaves out because its kernels are in the other spans). */
int vs_timer_read_kernel(const char* kernel, double* total_ms, int64_t* launches);
/* The same, plus the summed share of their passes' database tiles that those
 * spans covered (a filter pass's launches cover unequal parts: its list
 * launch a quarter chunk or 1/8 of a split pass; bench.py's roofline work). */
int vs_timer_read_kernel_share(const char* kernel, double* total_ms, int64_t* launches,
                               double* share);
/* Name of the fused search kernel the last search launched ("gemm_topk_x1",
 * "gemm_topk", "skinny_topk" or "gemv_topk"). */
const char* vs_timer_kernel(void);

#ifdef __cplusplus
}
#endif

#endif /* VSEARCH_H */
