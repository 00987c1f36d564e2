"""GPU, BASELINE config C3 at full size: 10M x 1536 fp32, k = 10, inner product
(and L2), the DEFAULT engine, batch 4096 and batch 1 — the headline workload
(bench.py) checked against the oracle on sampled queries from the first and
last query tiles.

Oracle at this size (chunked, tests only): the rows are read back from the
index (vs_reconstruct_n is bit-exact, test_gpu_parity.py) in 1M-row chunks;
numpy's fp32 sgemm pre-selects each sampled query's 64 best rows, the margin
between the 10th and the 64th is checked against the worst-case fp32 sgemm
error (gamma(d) * |q| * max|x|), so the candidate set provably holds the exact
top-10, and the candidates are rescored in fp64 (oracle/flat.py exact_scores,
faiss_order).  Acceptance as everywhere: labels exact except documented ties,
scores within 1e-5 relative."""

import numpy as np
import pytest

from oracle import flat

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N, D_, K = 10_000_000, 1536, 10
SAMPLE = [0, 1, 255, 256, 2047, 3839, 3840, 4095]  # first / last 256-query tiles


@pytest.fixture(scope="module")
def c3():
    from vsearch import _lib
    from vsearch import faiss as vfaiss
    from vsearch.synth import synthetic_rows

    assert _lib.device_count() >= 1
    xq = synthetic_rows(50_000_000, 4096, D_, 5678)
    out = {}
    for metric in (flat.METRIC_INNER_PRODUCT, flat.METRIC_L2):
        index = vfaiss.IndexFlat(D_, metric)
        index.reserve(N)
        index.add_synthetic(N, seed=1234)
        Db, Ib = index.search(xq, K)  # batch 4096 (default engine)
        D1, I1 = index.search(xq[SAMPLE[-1]:SAMPLE[-1] + 1], K)  # batch 1
        cand = _candidates(index, xq[SAMPLE], metric)
        out[metric] = (Db, Ib, D1, I1, cand)
        del index
    return xq, out


def _candidates(index, xs, metric, m=64, chunk=1_000_000):
    """Per sampled query: the m best rows by fp32 sgemm, with their fp64 exact
    scores, and the proof margin (the true top-K is inside the m)."""
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
        res.append((ids, exact))
    return res


def _oracle_topk(ids, exact, metric):
    key = exact if metric == flat.METRIC_L2 else -exact
    sel = flat.faiss_order(ids.astype(np.int64), key, K, metric)
    pos = {int(i): j for j, i in enumerate(ids)}
    return sel, np.array([exact[pos[int(i)]] for i in sel])


def _assert_parity(D, I, ref_i, ref_s, metric, qn2=0.0):
    for j in range(K):
        tol = 1e-5 * max(1.0, abs(ref_s[j]), 2200.0 if metric == flat.METRIC_L2 else 0.0)
        assert abs(float(D[j]) - ref_s[j]) <= tol, (j, D[j], ref_s[j])
        if I[j] != ref_i[j]:  # a different label only as a documented tie
            assert abs(float(D[j]) - ref_s[j]) <= tol, (j, I[j], ref_i[j])
    assert len(set(I.tolist())) == K


@pytest.mark.parametrize("metric", [flat.METRIC_INNER_PRODUCT, flat.METRIC_L2])
def test_c3_batch4096_sampled_against_oracle(c3, metric):
    xq, out = c3
    Db, Ib, _, _, cand = out[metric]
    assert Ib.shape == (4096, K)
    assert (Ib >= 0).all() and (Ib < N).all()
    diffs = np.diff(Db, axis=1)
    assert (diffs <= 0).all() if metric == flat.METRIC_INNER_PRODUCT else (diffs >= 0).all()
    for row, q in enumerate(SAMPLE):
        ref_i, ref_s = _oracle_topk(*cand[row], metric)
        _assert_parity(Db[q], Ib[q], ref_i, ref_s, metric)


@pytest.mark.parametrize("metric", [flat.METRIC_INNER_PRODUCT, flat.METRIC_L2])
def test_c3_batch1_against_oracle(c3, metric):
    xq, out = c3
    _, Ib, D1, I1, cand = out[metric]
    ref_i, ref_s = _oracle_topk(*cand[len(SAMPLE) - 1], metric)
    _assert_parity(D1[0], I1[0], ref_i, ref_s, metric)
    # batch 1 (HBM-bound kernel) and batch 4096 agree on the same query
    assert (I1[0] == Ib[SAMPLE[-1]]).all() or metric == flat.METRIC_L2
