"""Test doubles built on the CPU oracle (test infrastructure only).

OracleIndex implements the faiss-index surface that the host logic (LangChain
store, persistence, sharding) uses, with the oracle as its arithmetic, so the
host logic is testable on CPU.  It is never used by product code."""

from __future__ import annotations

import numpy as np

from oracle import flat


class OracleIndex:
    is_trained = True

    def __init__(self, d: int, metric: int = flat.METRIC_L2):
        self.d = int(d)
        self.metric_type = int(metric)
        self._x = np.zeros((0, self.d), dtype=np.float32)
        self._base = 0
        self.device = 0

    @property
    def ntotal(self) -> int:
        return self._x.shape[0]

    def add(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.shape[1] == self.d
        self._x = np.concatenate([self._x, x])

    def search(self, x, k, raw=False):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert x.shape[1] == self.d
        assert k > 0
        if raw:  # VS_RAW_ORDER: lexicographic (key, label), no IP tie rule
            D, I = flat.knn_lex(self._x, x, k, self.metric_type)
        else:
            D, I = flat.knn_exact(self._x, x, k, self.metric_type)
        I = np.where(I >= 0, I + self._base, -1)
        return D, I

    def reconstruct(self, i):
        if not 0 <= i < self.ntotal:
            raise RuntimeError("key out of range")
        return self._x[i].copy()

    def reconstruct_n(self, n0=0, ni=-1):
        if ni == -1:
            ni = self.ntotal - n0
        return self._x[n0:n0 + ni].copy()

    def remove_ids(self, ids):
        ids = np.asarray(ids, dtype=np.int64) - self._base
        self._x, n = flat.remove_ids(self._x, ids)
        return n

    def set_id_base(self, base):
        self._base = int(base)

    def reset(self):
        self._x = np.zeros((0, self.d), dtype=np.float32)


def oracle_merge(Dall, Iall, metric, k):
    """Merge gathered shard lists [G][nq][k_in] with the oracle's tie rule."""
    G, nq, kin = Dall.shape
    D = np.full((nq, k), flat.neutral(metric), dtype=np.float32)
    I = np.full((nq, k), -1, dtype=np.int64)
    for q in range(nq):
        s = Dall[:, q, :].ravel()
        ids = Iall[:, q, :].ravel()
        keep = ids >= 0
        s, ids = s[keep], ids[keep]
        if ids.size == 0:
            continue
        key = s if metric == flat.METRIC_L2 else -s
        sel = flat.faiss_order(ids, key, k, metric)
        pos = {int(i): j for j, i in enumerate(ids)}
        D[q, :sel.size] = [s[pos[int(i)]] for i in sel]
        I[q, :sel.size] = sel
    return D, I


def assert_against_candidates(D, I, cand, metric, k, d, strict):
    """One query's result (D, I) against its proven candidate set cand =
    (ids, fp64 scores, fp64 |x|^2, |q|^2): a set that provably holds the exact
    top-k (every other row strictly worse).  Every returned label must be a
    candidate, D[j] within the window of ITS OWN exact score, and a label that
    differs from the oracle's j-th only inside both windows (a tie).  Window:
    strict = the rounding of an exactly rescored key (flat.key_window), else the
    north star's fp32 contract (flat.score_tolerance)."""
    ids, exact, xn2, qn2 = cand
    pos = {int(i): j for j, i in enumerate(ids)}
    key = exact if metric == flat.METRIC_L2 else -exact
    ref_i = flat.faiss_order(np.asarray(ids, dtype=np.int64), key, k, metric)
    assert len(set(np.asarray(I).tolist())) == k

    def window(r):
        p = pos[int(r)]
        if strict:
            return float(flat.key_window(metric, exact[p], qn2, xn2[p], d))
        return float(flat.score_tolerance(metric, exact[p], qn2, xn2[p]))

    for j in range(k):
        assert int(I[j]) in pos, (j, int(I[j]), "not among the proven candidates")
        s_got = exact[pos[int(I[j])]]
        assert abs(float(D[j]) - s_got) <= window(I[j]), (j, int(I[j]), float(D[j]), s_got,
                                                          window(I[j]))
        if I[j] != ref_i[j]:
            s_ref = exact[pos[int(ref_i[j])]]
            assert abs(s_got - s_ref) <= window(I[j]) + window(ref_i[j]), (
                j, int(I[j]), int(ref_i[j]), s_got, s_ref)


def proven_candidates(index, xs, metric, N, K, m=64, chunk=1_000_000):
    """Per query of xs: the m best of the index's N rows (read back in chunks by
    reconstruct_n, bit-exact) by fp32 sgemm, with their fp64 exact scores and
    norms.  The margin between the K-th and the m-th sgemm score is checked
    against the worst-case fp32 sgemm error (gamma(d) |q| max|x|), so the set
    provably holds the exact top-K.  Returns (ids, exact, |x|^2, |q|^2) per
    query (the form assert_against_candidates takes)."""
    D_ = xs.shape[1]
    nq = xs.shape[0]
    best_s = np.full((nq, 0), -np.inf, np.float32)
    best_i = np.zeros((nq, 0), np.int64)
    xmax = 0.0
    rows = {}
    for r0 in range(0, N, chunk):
        xb = index.reconstruct_n(r0, min(chunk, N - r0))
        xmax = max(xmax, float(np.sqrt(np.einsum("ij,ij->i", xb, xb, dtype=np.float64).max())))
        s = xs @ xb.T  # fp32 sgemm
        if metric == flat.METRIC_L2:  # larger = better: 2 q.x - |x|^2 (|q|^2 is constant)
            s = 2.0 * s - np.einsum("ij,ij->i", xb, xb, dtype=np.float64)[None, :]
        s = np.asarray(s, np.float32)
        allv = np.concatenate([best_s, s], axis=1)
        alli = np.concatenate([best_i, np.broadcast_to(np.arange(r0, r0 + xb.shape[0]), s.shape)],
                              axis=1)
        part = np.argpartition(-allv, m - 1, axis=1)[:, :m]
        best_s = np.take_along_axis(allv, part, axis=1)
        best_i = np.take_along_axis(alli, part, axis=1)
        for q in range(nq):  # keep the candidate rows for the exact rescoring
            for r in best_i[q]:
                if r0 <= r < r0 + xb.shape[0]:
                    rows[int(r)] = xb[r - r0].copy()
    res = []
    u = 2.0 ** -24
    gam = D_ * u / (1 - D_ * u)
    for q in range(nq):
        ids = best_i[q]
        order = np.argsort(-best_s[q], kind="stable")
        s_sorted = best_s[q][order]
        qn = float(np.sqrt(np.dot(xs[q].astype(np.float64), xs[q].astype(np.float64))))
        bound = 2.0 * gam * qn * xmax * (2.0 if metric == flat.METRIC_L2 else 1.0) + 1e-3
        # fp32 preselection can only be wrong inside this margin
        assert s_sorted[K - 1] - s_sorted[m - 1] > 2 * bound, (q, s_sorted[K - 1], s_sorted[-1])
        xb = np.stack([rows[int(r)] for r in ids])
        exact = flat.exact_scores(xb, xs[q:q + 1], metric)[0]
        xn2 = np.einsum("ij,ij->i", xb.astype(np.float64), xb.astype(np.float64))
        res.append((ids, exact, xn2, qn * qn))
    return res
