"""GPU, BASELINE configs C2 and C4 at full size with the DEFAULT engine (the
staged int8 -> bf16 -> fp32 filter-and-verify path), checked against the fp64
oracle on 64 sampled queries / students spanning every query tile and the
self-join's 65,536-row chunks.

C2: 1M x 1536 fp32, batch 1024, top-10 inner product (bench.py --workload c2).
C4: 1M x 1536 fp32, cosine top-50 self-join excluding self (bench.py --workload
c4, graph_refresher/main.py:339-354 at 1M students).  The rows are read back
from the index (vs_reconstruct_n is bit-exact) and scored in fp64
(oracle/flat.py).  Acceptance: STRICT (the staged engine's keys are fp64
rescorings rounded once): every D is within the rounding window of its own
label's exact score (oracle/flat.py key_window) and a label differs from the
oracle's only when the two exact scores lie within both windows."""

import numpy as np
import pytest

from helpers import assert_against_candidates
from oracle import flat

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N, D_ = 1_000_000, 1536


def _rows(index, chunk=250_000):
    return np.concatenate([index.reconstruct_n(r0, min(chunk, N - r0))
                           for r0 in range(0, N, chunk)])


def test_c2_batch1024_sampled_against_oracle():
    from vsearch import faiss as vfaiss
    from vsearch.synth import synthetic_rows

    k = 10
    index = vfaiss.IndexFlatIP(D_)
    index.add_synthetic(N, seed=1234)
    xq = synthetic_rows(50_000_000, 1024, D_, 5678)
    D, I = index.search(xq, k)
    assert I.shape == (1024, k) and (I >= 0).all() and (I < N).all()
    assert (np.diff(D, axis=1) <= 0).all()
    # 64 queries: 16 per query tile, both ends of each
    sample = sorted({q for t in range(4) for q in [256 * t + j for j in range(0, 256, 17)]
                     + [256 * t + 255]})
    xb = _rows(index)
    s = np.zeros((len(sample), N))
    q64 = xq[sample].astype(np.float64)
    for r0 in range(0, N, 250_000):
        s[:, r0:r0 + 250_000] = q64 @ xb[r0:r0 + 250_000].astype(np.float64).T
    xn2 = np.einsum("ij,ij->i", xb.astype(np.float64), xb.astype(np.float64))
    for row, q in enumerate(sample):
        top = np.argpartition(-s[row], 64)[:64]  # the exact 64 best: a proven candidate set
        cand = (top.astype(np.int64), s[row, top], xn2[top], float(q64[row] @ q64[row]))
        assert_against_candidates(D[q], I[q], cand, flat.METRIC_INNER_PRODUCT, k, D_, strict=True)


def test_c4_selfjoin_top50_sampled_against_oracle():
    from vsearch import faiss as vfaiss

    k = 50
    index = vfaiss.IndexFlatIP(D_)
    index.add_synthetic(N, seed=4321)
    S, I = index.selfjoin(k)
    assert I.shape == (N, k) and (I >= 0).all() and (I < N).all()
    assert not (I == np.arange(N)[:, None]).any()
    # 64 students: both sides of every 65,536-row chunk boundary and of query
    # tiles inside chunks, plus the last rows
    edges = [c * 65536 + o for c in range(16) for o in (-1, 0)] + [255, 256, 500000, 999743]
    fill = np.linspace(1, N - 2, 64 - len(edges)).astype(np.int64).tolist()
    sample = np.array(sorted({e for e in edges + fill + [N - 1] if 0 <= e < N}))
    xb = _rows(index)
    Sr, Ir = flat.pgvector_cosine_topk(xb, k, q_rows=sample)
    bad = flat.selfjoin_mismatches(S[sample], I[sample], Sr, Ir, xb, sample, strict=True)
    assert not bad, bad[:5]
