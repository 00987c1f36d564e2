"""ORACLE — test infrastructure only.  CPU restatement of the reference's hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker (or the timed CPU baseline) — never as the
thing measured or shipped.

What it restates
  faiss-cpu 1.11.0 ``IndexFlat::search`` (pinned at /root/reference/poetry.lock:866-867;
  the package is NOT vendored in /root/reference and is not installable here), as
  reached through LangChain's ``FAISS.similarity_search_with_score_by_vector``
  (call sites: src/recommendation_api/mcp_book_server.py:142,
  candidate_builder.py:187,321, service.py:529,627):
    * exact k nearest rows, squared L2 ascending (IndexFlatL2, the LangChain
      default: SURVEY.md §0.2) or inner product descending (IndexFlatIP);
    * ties broken by the lower label (heap ``CMax/CMin::cmp2`` + strict admission
      in increasing-label scan order);
    * k > ntotal padded with label -1 and the heap's neutral value
      (``std::numeric_limits<float>::max()`` / ``lowest()``, i.e. +/-FLT_MAX);
    * BLAS branch for nq >= 20: dis = |x|^2 + |y|^2 - 2<x,y>, clamped at 0;
      sequential branch for nq < 20: dis = sum (x - y)^2.
  faiss ``IndexFlat::remove_ids(IDSelectorBatch)``: stable compaction.
  pgvector ``<=>`` (image ankane/pgvector:latest, docker-compose.yml:16, unpinned)
  as used by src/graph_refresher/main.py:339-354: cosine similarity
  dot/sqrt(|a|^2 |b|^2), exclude self, top-k, then ``sim >= threshold``.

Parity status: faiss/langchain/pgvector cannot be imported or compiled here
 and the reference's tests pin no ids or scores.  This oracle is
pinned to the hand-derived known answers of the reference's own fixtures (the
3-d ``[i%3]*3`` embedding stub and ``[0,0,0]`` query,
tests/test_integration_ingestion_graph.py:40-48) and to golden vectors generated
from data/*.csv (tests/golden/, script committed).  Everything beyond that is
"parity unpinned" with respect to faiss itself.
"""

from __future__ import annotations

import numpy as np

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
FLT_MAX = np.float32(np.finfo(np.float32).max)


def round_bf16(x) -> np.ndarray:
    """float32 -> nearest-even bf16 -> float32 (what a bf16 index stores)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    nan = np.isnan(np.asarray(x, dtype=np.float32))
    out = r.astype(np.uint32).view(np.float32)
    out = np.where(nan, np.float32(np.nan), out)
    return out.astype(np.float32)


def neutral(metric: int) -> np.float32:
    """faiss heap neutral value: CMax -> FLT_MAX (L2), CMin -> lowest (IP)."""
    return FLT_MAX if metric == METRIC_L2 else -FLT_MAX


def exact_scores(xb: np.ndarray, xq: np.ndarray, metric: int) -> np.ndarray:
    """fp64 scores (nq, n): squared L2 or inner product."""
    xb64 = np.asarray(xb, dtype=np.float64)
    xq64 = np.asarray(xq, dtype=np.float64)
    ip = xq64 @ xb64.T
    if metric == METRIC_INNER_PRODUCT:
        return ip
    nb = np.einsum("ij,ij->i", xb64, xb64)
    nqn = np.einsum("ij,ij->i", xq64, xq64)
    d = nqn[:, None] + nb[None, :] - 2.0 * ip
    return np.maximum(d, 0.0)


def faiss_order(cand: np.ndarray, key: np.ndarray, k: int, metric: int) -> np.ndarray:
    """Labels faiss's heap returns, in output order, from candidates (label, key)
    where key is the distance (L2) or the negated score (IP), smaller = better.

    L2 (CMax heap, cmp2 prefers the larger label at the top): the k best by
    (key, label); output ascending by (key, label).
    IP (CMin heap, cmp2 prefers the SMALLER label at the top): with v the k-th key,
    c the count strictly better, a_0 < a_1 < ... the labels with key v, and g_i the
    number of strictly-better labels below a_i, the scan admits a_i while
    i + g_i < k (|A| of them) and later better rows evict the smallest admitted
    labels first, so a_{|A|-r} .. a_{|A|-1} stay (r = k - c).  heap_reorder then
    emits ascending key with DESCENDING label inside equal keys.
    (Derived statement by statement from faiss/utils/Heap.h + ordered_key_value.h;
    pinned against the C restatement oracle/faiss_flat.c in tests.)"""
    order = np.lexsort((cand, key))
    cand, key = cand[order], key[order]
    if metric == METRIC_L2:
        return cand[:k]
    if cand.size > k:
        v = key[k - 1]
        c = int(np.count_nonzero(key < v))
        run = cand[c:][key[c:] == v]
        better = np.sort(cand[:c])
        g = np.searchsorted(better, run)
        A = int(np.count_nonzero(np.arange(run.size) + g < k))
        r = k - c
        cand = np.concatenate([cand[:c], run[A - r:A]])
        key = np.concatenate([key[:c], np.full(r, v, dtype=key.dtype)])
    # descending label inside equal keys
    order = np.lexsort((-cand, key))
    return cand[order]


def select_topk(scores: np.ndarray, k: int, metric: int, valid: np.ndarray | None = None,
                rule: str = "faiss"):
    """Top-k per row with faiss's admission (a value equal to the neutral, or
    NaN, never enters) and faiss's tie rule (rule="faiss") or plain
    (score, lower label) order (rule="lex", used for pgvector / SQL where tie
    order is unspecified).  Returns (D float32, I int64) padded with (neutral, -1)."""
    nq, n = scores.shape
    D = np.full((nq, k), neutral(metric), dtype=np.float32)
    I = np.full((nq, k), -1, dtype=np.int64)
    key = scores if metric == METRIC_L2 else -scores
    lim = float(FLT_MAX)
    for q in range(nq):
        kq = key[q]
        with np.errstate(invalid="ignore"):
            ok = np.isfinite(kq) & (kq < lim)
        if valid is not None:
            ok &= valid[q]
        cand = np.nonzero(ok)[0]
        if cand.size == 0:
            continue
        kk = kq[cand]
        if cand.size > k:
            part = np.argpartition(kk, k - 1)[:k]
            thr = kk[part].max()
            sel = np.nonzero(kk <= thr)[0]
            cand, kk = cand[sel], kk[sel]
        if rule == "faiss":
            ids = faiss_order(cand.astype(np.int64), kk, k, metric)
        else:
            ids = cand[np.lexsort((cand, kk))][:k]
        m = ids.size
        I[q, :m] = ids
        D[q, :m] = scores[q, ids].astype(np.float32)
    return D, I


def knn_exact(xb, xq, k: int, metric: int):
    """Reference semantics with fp64 arithmetic (the parity yardstick)."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    if xb.shape[0] == 0:
        return (np.full((xq.shape[0], k), neutral(metric), np.float32),
                np.full((xq.shape[0], k), -1, np.int64))
    return select_topk(exact_scores(xb, xq, metric), k, metric)


def knn_lex(xb, xq, k: int, metric: int):
    """The k lexicographically best (key, label) rows, in that order, fp64
    scores: what libvsearch returns under VS_RAW_ORDER (one shard's half of an
    exact sharded search; faiss_order then reproduces faiss on the union)."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    if xb.shape[0] == 0:
        return (np.full((xq.shape[0], k), neutral(metric), np.float32),
                np.full((xq.shape[0], k), -1, np.int64))
    return select_topk(exact_scores(xb, xq, metric), k, metric, rule="lex")


def knn_faiss_fp32(xb, xq, k: int, metric: int, bs_x: int = 4096, bs_y: int = 65536):
    """faiss's fp32 arithmetic (BLAS branch): blocked sgemm + norms + clamp + a
    running top-k per query.  Used as the timed CPU baseline (kind "port"):
    the sgemm is numpy's multithreaded BLAS, like faiss's own sgemm call.
    Ties inside a block are resolved by label like faiss's heap."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq, n = xq.shape[0], xb.shape[0]
    D = np.full((nq, k), neutral(metric), dtype=np.float32)
    I = np.full((nq, k), -1, dtype=np.int64)
    if n == 0:
        return D, I
    qn = np.einsum("ij,ij->i", xq, xq, dtype=np.float32) if metric == METRIC_L2 else None
    bn = np.einsum("ij,ij->i", xb, xb, dtype=np.float32) if metric == METRIC_L2 else None
    for i0 in range(0, nq, bs_x):
        i1 = min(nq, i0 + bs_x)
        keyk = np.full((i1 - i0, k), np.inf, dtype=np.float32)
        idk = np.full((i1 - i0, k), -1, dtype=np.int64)
        for j0 in range(0, n, bs_y):
            j1 = min(n, j0 + bs_y)
            ip = xq[i0:i1] @ xb[j0:j1].T
            if metric == METRIC_L2:
                blk = (qn[i0:i1, None] + bn[None, j0:j1]) - np.float32(2.0) * ip
                np.maximum(blk, np.float32(0.0), out=blk)
            else:
                blk = -ip
            kk = np.concatenate([keyk, blk], axis=1)
            ii = np.concatenate([idk, np.broadcast_to(np.arange(j0, j1), blk.shape)], axis=1)
            m = min(k, kk.shape[1])
            part = np.argpartition(kk, m - 1, axis=1)[:, :m]
            keyk = np.take_along_axis(kk, part, axis=1)
            idk = np.take_along_axis(ii, part, axis=1)
        order = np.lexsort((idk, keyk), axis=1)
        keyk = np.take_along_axis(keyk, order, axis=1)
        idk = np.take_along_axis(idk, order, axis=1)
        fill = idk >= 0
        sc = keyk if metric == METRIC_L2 else -keyk
        D[i0:i1] = np.where(fill, sc, neutral(metric))
        I[i0:i1] = np.where(fill, idk, -1)
    return D, I


def score_tolerance(metric: int, s_ref, xq_norm2=0.0, xb_norm2=0.0):
    """The fp32 contract of the north star: 1e-5 relative with an absolute floor
    of 1e-5.  For squared L2 through the norm expansion the magnitude that sets
    fp32 rounding is |q|^2 + |x|^2 (the terms that cancel), so it enters the scale."""
    scale = np.maximum(1.0, np.abs(s_ref))
    if metric == METRIC_L2:
        scale = np.maximum(scale, np.asarray(xq_norm2) + np.asarray(xb_norm2))
    return 1e-5 * scale


U32 = 2.0 ** -24  # unit roundoff of fp32


def key_window(metric: int, s, qn2, xn2, d: int, cosine: bool = False):
    """How far an engine key that is the fp32 ROUNDING of an exactly computed
    score can sit from the fp64 score s (the filter-and-verify engine: fp64 sums
    of the fp32 products, rounded once; vs_gemm_x1.hip exact_key; fp64-summed
    norms, vs_support.hip row_norms_kernel):
      IP      key = fl(s):                          U|s|
      L2      key = fl(fl(fl(|q|^2) + fl(|x|^2)) - 2 fl(s)), clamped at 0:
              every rounding acts on at most 2(|q|^2 + |x|^2):  5U(|q|^2 + |x|^2)
      cosine  key = fl(fl(s) * fl(fl(1/|q|) * fl(1/|x|))): 6U|sim|
    (taken as 6U / 8U), plus the fp64 sum's own d * 2^-52 |q||x|.  Two rows can
    come out in either order only when their windows overlap: that is the tie
    window the strict checks use (instead of the fp32 contract's 1e-5)."""
    s = np.abs(np.asarray(s, dtype=np.float64))
    qn2 = np.asarray(qn2, dtype=np.float64)
    xn2 = np.asarray(xn2, dtype=np.float64)
    floor = d * 2.0 ** -52 * np.sqrt(qn2 * xn2) + 1e-300
    if cosine:
        return 8 * U32 * s + d * 2.0 ** -52 + 1e-300
    if metric == METRIC_L2:
        return 6 * U32 * (qn2 + xn2) + 4 * floor
    return U32 * s + floor


def mismatches(D, I, Dr, Ir, metric: int, xb, xq, rtol: float = 1e-5, strict: bool = False):
    """Parity check of a (D, I) result against the fp64 oracle result (Dr, Ir).

    * every returned label is valid and unique per query, -1 exactly where the
      oracle pads;
    * D[q, j] within tolerance of the exact score of the returned label;
    * the returned label's exact score within tolerance of the oracle's j-th
      score (a different label is accepted only as a documented tie);
    Tolerance: the north star's fp32 contract (1e-5 relative; for squared L2
    the scale includes |q|^2 + |x|^2), or with ``strict`` the rounding window of
    an exactly rescored key (key_window): D must be the fp32 rounding of the
    label's exact score, and a different label is a tie only when the two exact
    scores are within both windows — what the filter-and-verify engine proves.
    Returns a list of human-readable problems (empty = parity)."""
    xb = np.asarray(xb, dtype=np.float32)
    xq = np.asarray(xq, dtype=np.float32)
    D = np.asarray(D)
    I = np.asarray(I)
    bad = []
    nq, k = Ir.shape
    nb2 = np.einsum("ij,ij->i", xb.astype(np.float64), xb.astype(np.float64))
    nq2 = np.einsum("ij,ij->i", xq.astype(np.float64), xq.astype(np.float64))
    for q in range(nq):
        ids = I[q]
        real = ids[ids >= 0]
        if len(set(real.tolist())) != real.size:
            bad.append((q, "duplicate labels", ids.tolist()))
            continue
        if not np.array_equal(ids < 0, Ir[q] < 0):
            bad.append((q, "padding differs", ids.tolist(), Ir[q].tolist()))
            continue
        if np.any(ids >= xb.shape[0]):
            bad.append((q, "label out of range", ids.tolist()))
            continue
        for j in range(k):
            if ids[j] < 0:
                if D[q, j] != neutral(metric):
                    bad.append((q, j, "padding score", float(D[q, j])))
                continue
            s_got = exact_scores(xb[ids[j]:ids[j] + 1], xq[q:q + 1], metric)[0, 0]
            if strict:
                tol = float(key_window(metric, s_got, nq2[q], nb2[ids[j]], xb.shape[1]))
            else:
                tol = score_tolerance(metric, s_got, nq2[q], nb2[ids[j]]) * (rtol / 1e-5)
            if abs(float(D[q, j]) - s_got) > tol:
                bad.append((q, j, "score", float(D[q, j]), float(s_got), float(tol)))
            if ids[j] != Ir[q, j]:
                s_ref = exact_scores(xb[Ir[q, j]:Ir[q, j] + 1], xq[q:q + 1], metric)[0, 0]
                if strict:
                    tol2 = tol + float(key_window(metric, s_ref, nq2[q], nb2[Ir[q, j]], xb.shape[1]))
                else:
                    tol2 = score_tolerance(metric, s_ref, nq2[q], nb2[Ir[q, j]]) * (rtol / 1e-5)
                if abs(s_got - s_ref) > tol2:
                    bad.append((q, j, "label", int(ids[j]), int(Ir[q, j]), s_got, s_ref, tol2))
    return bad


def selfjoin_mismatches(S, I, Sr, Ir, x, q_rows, strict: bool = False):
    """Self-join check (pgvector cosine, exclude self) of (S, I) against the
    oracle's (Sr, Ir) for query rows q_rows of x: labels equal except ties,
    similarities within 1e-5 absolute, or with ``strict`` within the cosine
    key window (key_window) of the returned label's exact similarity."""
    x64 = np.asarray(x, dtype=np.float64)
    nrm = np.sqrt(np.einsum("ij,ij->i", x64, x64))
    d = x64.shape[1]
    bad = []
    for row, q in enumerate(np.asarray(q_rows)):
        for j in range(I.shape[1]):
            a, b = int(I[row, j]), int(Ir[row, j])
            if (a < 0) != (b < 0):
                bad.append((row, j, "padding", a, b))
                continue
            if a < 0:
                continue
            s_got = float(x64[q] @ x64[a]) / (nrm[q] * nrm[a])
            tol = float(key_window(0, s_got, 0, 0, d, cosine=True)) if strict else 1e-5
            if abs(float(S[row, j]) - s_got) > tol:
                bad.append((row, j, "sim", float(S[row, j]), s_got, tol))
            if a != b:
                s_ref = float(x64[q] @ x64[b]) / (nrm[q] * nrm[b])
                tol2 = tol + float(key_window(0, s_ref, 0, 0, d, cosine=True)) if strict else 1e-5
                if abs(s_got - s_ref) > tol2 or a == int(q):
                    bad.append((row, j, "label", a, b, s_got, s_ref))
    return bad


def remove_ids(xb: np.ndarray, ids) -> tuple[np.ndarray, int]:
    """faiss IndexFlat::remove_ids(IDSelectorBatch): keep rows not selected, in order."""
    ids = np.asarray(ids, dtype=np.int64).ravel()
    n = xb.shape[0]
    sel = np.zeros(n, dtype=bool)
    inr = ids[(ids >= 0) & (ids < n)]
    sel[inr] = True
    return xb[~sel], int(sel.sum())


def pgvector_cosine_topk(x, k: int, q_rows=None, exclude_self: bool = True,
                         min_sim: float | None = None):
    """Student self-join (graph_refresher/main.py:339-354), fp64:
    sim = dot / sqrt(|a|^2 |b|^2); zero-norm rows give NaN and never match;
    top-k by similarity (ties: lower row), then sim >= min_sim."""
    x64 = np.asarray(x, dtype=np.float64)
    n = x64.shape[0]
    q_rows = np.arange(n) if q_rows is None else np.asarray(q_rows)
    nrm = np.einsum("ij,ij->i", x64, x64)
    with np.errstate(divide="ignore", invalid="ignore"):
        sims = (x64[q_rows] @ x64.T) / np.sqrt(nrm[q_rows, None] * nrm[None, :])
    valid = np.ones_like(sims, dtype=bool)
    if exclude_self:
        valid[np.arange(q_rows.size), q_rows] = False
    S, I = select_topk(sims, k, METRIC_INNER_PRODUCT, valid=valid, rule="lex")
    if min_sim is not None:
        drop = ~(S >= np.float32(min_sim)) | (I < 0)
        S[drop] = -FLT_MAX
        I[drop] = -1
    return S, I


def mismatches_vec(D, I, Dr, Ir, metric: int, xb, xq, rtol: float = 1e-5, qchunk: int = 128):
    """mismatches() for large k, vectorised (the fp32 contract only): the same
    checks — unique valid labels, padding where the oracle pads, D within
    tolerance of the returned label's exact score, a label other than the
    oracle's j-th only within both tolerances (a tie) — on numpy arrays in
    query chunks.  Returns a list of problems (empty = parity)."""
    xb64 = np.asarray(xb, dtype=np.float64)
    xq64 = np.asarray(xq, dtype=np.float64)
    D = np.asarray(D)
    I = np.asarray(I)
    Ir = np.asarray(Ir)
    nb2 = np.einsum("ij,ij->i", xb64, xb64)
    nq2 = np.einsum("ij,ij->i", xq64, xq64)
    bad = []
    if np.any(I >= xb64.shape[0]):
        return [("label out of range",)]
    pad = (I < 0) != (Ir < 0)
    if pad.any():
        q = int(np.nonzero(pad.any(axis=1))[0][0])
        return [(q, "padding differs", I[q].tolist(), Ir[q].tolist())]
    srt = np.sort(np.where(I >= 0, I, -np.arange(1, I.shape[1] + 1)[None, :]), axis=1)
    dup = (np.diff(srt, axis=1) == 0).any(axis=1)
    if dup.any():
        return [(int(np.nonzero(dup)[0][0]), "duplicate labels")]
    empty = I < 0
    if np.any(D[empty] != neutral(metric)):
        return [("padding score",)]

    def scores(ids, q0, q1):
        safe = np.where(ids >= 0, ids, 0)
        ip = np.einsum("qd,qkd->qk", xq64[q0:q1], xb64[safe])
        if metric == METRIC_INNER_PRODUCT:
            return ip
        return np.maximum(nq2[q0:q1, None] + nb2[safe] - 2.0 * ip, 0.0)

    def tol(s, ids, q0, q1):
        scale = np.maximum(1.0, np.abs(s))
        if metric == METRIC_L2:
            scale = np.maximum(scale, nq2[q0:q1, None] + nb2[np.where(ids >= 0, ids, 0)])
        return 1e-5 * scale * (rtol / 1e-5)

    for q0 in range(0, I.shape[0], qchunk):
        q1 = min(I.shape[0], q0 + qchunk)
        ids, rids = I[q0:q1], Ir[q0:q1]
        valid = ids >= 0
        s_got = scores(ids, q0, q1)
        t_got = tol(s_got, ids, q0, q1)
        off = valid & (np.abs(D[q0:q1].astype(np.float64) - s_got) > t_got)
        for q, j in zip(*np.nonzero(off)):
            bad.append((q0 + int(q), int(j), "score", float(D[q0 + q, j]), float(s_got[q, j])))
        diff = valid & (ids != rids)
        if diff.any():
            s_ref = scores(rids, q0, q1)
            t_ref = tol(s_ref, rids, q0, q1)
            lab = diff & (np.abs(s_got - s_ref) > t_got + t_ref)
            for q, j in zip(*np.nonzero(lab)):
                bad.append((q0 + int(q), int(j), "label", int(ids[q, j]), int(rids[q, j]),
                            float(s_got[q, j]), float(s_ref[q, j])))
        if len(bad) > 20:
            break
    return bad
