"""GPU, BASELINE config C3 at full size: 10M x 1536 fp32, k = 10, inner product
(and L2), the DEFAULT engine, batch 4096 and batch 1 — the headline workload
(bench.py) checked against the oracle on 64 sampled queries spanning all 16 query tiles,
plus the embedding-like clustered corpus bench.py --data clustered measures
(unit-norm rows, 1024 centroids: the int8 -> bf16 -> deep bf16 hand-off).

Oracle at this size (chunked, tests only): the rows are read back from the
index (vs_reconstruct_n is bit-exact, test_gpu_parity.py) in 1M-row chunks;
numpy's fp32 sgemm pre-selects each sampled query's 64 best rows, the margin
between the 10th and the 64th is checked against the worst-case fp32 sgemm
error (gamma(d) * |q| * max|x|), so the candidate set provably holds the exact
top-10, and the candidates are rescored in fp64 (oracle/flat.py exact_scores,
faiss_order).

Acceptance, batch 4096 (the staged filter-and-verify engine, whose keys are
fp64 rescorings rounded once): STRICT — every returned label is one of the 64
proven candidates, D[q, j] is within the rounding window (oracle/flat.py
key_window) of that label's own fp64 score, and a label differing from the
oracle's j-th is accepted only when the two fp64 scores lie within both
windows (a true fp32-key tie).  Batch 1 (the HBM-bound GEMV, fp32 sums like
faiss's own fvec_inner_product): the north star's fp32 contract, 1e-5 of
max(1, |s|) (squared L2: of |q|^2 + |x|^2 of the pair)."""

import numpy as np
import pytest

from helpers import assert_against_candidates, proven_candidates
from oracle import flat

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N, D_, K = 10_000_000, 1536, 10
# 64 queries: the first and last query of every 256-query tile, two more inside
# each (every tile of the int8 pass, both ends of its lane lists' query blocks);
# the proven-candidate oracle's cost is the 61 GB read-back, not the sample size
SAMPLE = sorted({q for t in range(16) for q in (256 * t, 256 * t + 37, 256 * t + 160,
                                                 256 * t + 255)})
CL_SAMPLE = SAMPLE[::2] + [4095]  # clustered: 33 queries (m = 256 candidates each)
KW = (30, 60, 100)  # inner product's wide k (checked on the IP candidate sets, m = 256)
KW_L2 = (200,)  # L2 past one 64-entry page (the staged engine's 256 candidates)


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
        wide = {}
        # wide k at batch 4096 — the service's (service.py:627 k = 30, :529 k = 60:
        # 64 / 128 candidates per query) and past one page (the agent's k,
        # mcp_book_server.py:115,142: 256 candidates) — and at batch 1 (the skinny
        # int8 pass with the same candidate counts)
        kws = KW if metric == flat.METRIC_INNER_PRODUCT else KW_L2
        for kw in kws:
            wide[kw] = index.search(xq, kw)
            wide[(kw, 1)] = index.search(xq[SAMPLE[-1]:SAMPLE[-1] + 1], kw)
        cand = proven_candidates(index, xq[SAMPLE], metric, N, max(kws), m=256)
        out[metric] = (Db, Ib, D1, I1, cand, wide)
        del index
    return xq, out


@pytest.mark.parametrize("metric", [flat.METRIC_INNER_PRODUCT, flat.METRIC_L2])
def test_c3_batch4096_sampled_against_oracle(c3, metric):
    xq, out = c3
    Db, Ib, _, _, cand, _ = out[metric]
    assert Ib.shape == (4096, K)
    assert (Ib >= 0).all() and (Ib < N).all()
    diffs = np.diff(Db, axis=1)
    assert (diffs <= 0).all() if metric == flat.METRIC_INNER_PRODUCT else (diffs >= 0).all()
    for row, q in enumerate(SAMPLE):
        assert_against_candidates(Db[q], Ib[q], cand[row], metric, K, D_, strict=True)


@pytest.fixture(scope="module")
def c3_clustered():
    """bench.py's clustered corpus (ClusteredRows: normalize(c[i % 1024] + 0.5 n),
    seed 1234, queries noise seed 5678) at 10M x 1536, inner product: the data
    shape the reference's text-embedding-3-small vectors have (settings.py:16-18)
    and the case where most queries leave the int8 stage."""
    import torch

    from bench import ClusteredRows
    from vsearch import faiss as vfaiss

    index = vfaiss.IndexFlat(D_, flat.METRIC_INNER_PRODUCT)
    index.reserve(N)
    gen = ClusteredRows(torch, D_, seed=1234)
    for r0 in range(0, N, 1 << 20):
        x = gen.rows(r0, min(1 << 20, N - r0))
        index.add_device(x.data_ptr(), x.shape[0])
        torch.cuda.synchronize()
        del x
    xq = ClusteredRows(torch, D_, seed=1234, noise_seed=5678).rows(0, 4096).cpu().numpy()
    torch.cuda.empty_cache()
    D, I = index.search(xq, K)
    D2, I2 = index.search(xq, K)  # the adaptive order's second search (bf16 first)
    cand = proven_candidates(index, xq[CL_SAMPLE], flat.METRIC_INNER_PRODUCT, N, K, m=256)
    del index
    return D, I, D2, I2, cand


def test_c3_clustered_sampled_against_oracle(c3_clustered):
    D, I, D2, I2, cand = c3_clustered
    assert (I >= 0).all() and (I < N).all() and (np.diff(D, axis=1) <= 0).all()
    for row, q in enumerate(CL_SAMPLE):
        assert_against_candidates(D[q], I[q], cand[row], flat.METRIC_INNER_PRODUCT, K, D_,
                                  strict=True)
        assert_against_candidates(D2[q], I2[q], cand[row], flat.METRIC_INNER_PRODUCT, K, D_,
                                  strict=True)


@pytest.mark.parametrize("metric", [flat.METRIC_INNER_PRODUCT, flat.METRIC_L2])
def test_c3_batch1_against_oracle(c3, metric):
    xq, out = c3
    _, Ib, D1, I1, cand, _ = out[metric]
    assert_against_candidates(D1[0], I1[0], cand[len(SAMPLE) - 1], metric, K, D_, strict=False)
    # batch 1 (HBM-bound kernel) and batch 4096 agree on the same query
    assert (I1[0] == Ib[SAMPLE[-1]]).all() or metric == flat.METRIC_L2


@pytest.mark.parametrize("metric,kw", [(flat.METRIC_INNER_PRODUCT, k) for k in KW] +
                         [(flat.METRIC_L2, k) for k in KW_L2])
def test_c3_wide_k_against_oracle(c3, metric, kw):
    """Inner product k = 30, 60 and 100 (the filter pass with 64, 128 and 256
    candidates per query, faiss's tie rule over the 2k - 1 best) and L2 k = 200
    at batch 4096, and the same k at batch 1: strict on the sampled queries
    against their proven 256-row candidate sets."""
    xq, out = c3
    _, _, _, _, cand, wide = out[metric]
    D, I = wide[kw]
    assert I.shape == (4096, kw) and (I >= 0).all() and (I < N).all()
    diffs = np.diff(D, axis=1)
    assert (diffs <= 0).all() if metric == flat.METRIC_INNER_PRODUCT else (diffs >= 0).all()
    for row, q in enumerate(SAMPLE):
        assert_against_candidates(D[q], I[q], cand[row], metric, kw, D_, strict=True)
    D1, I1 = wide[(kw, 1)]
    assert_against_candidates(D1[0], I1[0], cand[len(SAMPLE) - 1], metric, kw, D_, strict=True)
