"""GPU: bf16 row storage (BASELINE config 5).

A bf16 index rounds rows and queries to bf16 (nearest even) and accumulates
products in fp32, so it is EXACT with respect to the rounded vectors (checked
against the fp64 oracle on round_bf16 inputs, same tolerance as fp32) and
APPROXIMATE with respect to the original fp32 vectors (reported as recall@k)."""

import numpy as np
import pytest

from oracle import flat

pytestmark = pytest.mark.gpu

L2, IP = flat.METRIC_L2, flat.METRIC_INNER_PRODUCT


@pytest.fixture(scope="module")
def vf():
    from vsearch import _lib
    from vsearch import faiss as vfaiss

    assert _lib.device_count() >= 1
    return vfaiss


def _rand(n, d, seed):
    return np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("nq", [1, 3, 8, 9, 40, 130])
@pytest.mark.parametrize("k", [1, 5, 10, 32])
def test_bf16_exact_on_rounded_vectors(vf, metric, nq, k):
    xb = _rand(2500, 200, 1)
    xq = _rand(nq, 200, 2)
    index = vf.IndexFlat(200, metric, dtype="bf16")
    index.add(xb)
    D, I = index.search(xq, k)
    rb, rq = flat.round_bf16(xb), flat.round_bf16(xq)
    Dr, Ir = flat.knn_exact(rb, rq, k, metric)
    bad = flat.mismatches(D, I, Dr, Ir, metric, rb, rq)
    assert not bad, bad[:5]


@pytest.mark.parametrize("d", [3, 64, 100, 1536])
def test_bf16_dims_and_reconstruct(vf, d):
    xb = _rand(300, d, 3)
    index = vf.IndexFlatL2(d, dtype="bf16")
    assert index.dtype == "bf16"
    index.add(xb)
    np.testing.assert_array_equal(index.reconstruct_n(0, 300), flat.round_bf16(xb))
    np.testing.assert_array_equal(index.reconstruct(299), flat.round_bf16(xb[299:]).ravel())
    xq = _rand(5, d, 4)
    D, I = index.search(xq, 7)
    rb, rq = flat.round_bf16(xb), flat.round_bf16(xq)
    Dr, Ir = flat.knn_exact(rb, rq, 7, L2)
    assert not flat.mismatches(D, I, Dr, Ir, L2, rb, rq)


def test_bf16_remove_and_add(vf):
    xb = _rand(5000, 64, 5)
    index = vf.IndexFlatIP(64, dtype="bf16")
    index.add(xb)
    rm = np.arange(0, 5000, 7, dtype=np.int64)
    assert index.remove_ids(rm) == rm.size
    xr, _ = flat.remove_ids(flat.round_bf16(xb), rm)
    np.testing.assert_array_equal(index.reconstruct_n(0, index.ntotal), xr)
    index.add(xb[:100])
    xr = np.concatenate([xr, flat.round_bf16(xb[:100])])
    xq = _rand(20, 64, 6)
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xr, flat.round_bf16(xq), 10, IP)
    assert not flat.mismatches(D, I, Dr, Ir, IP, xr, flat.round_bf16(xq))


def test_bf16_synthetic_matches_rounded_generator(vf):
    from vsearch.synth import synthetic_rows

    index = vf.IndexFlatIP(1536, dtype="bf16")
    index.add_synthetic(257, seed=1234, row0=123)
    np.testing.assert_array_equal(index.reconstruct_n(0, 257),
                                  flat.round_bf16(synthetic_rows(123, 257, 1536, 1234)))


@pytest.mark.parametrize("metric", [L2, IP])
def test_bf16_recall_vs_fp32(vf, metric):
    """recall@10 of the bf16 index against fp32 exact search (C5's reported metric)."""
    rng = np.random.default_rng(7)
    cent = rng.standard_normal((64, 256)).astype(np.float32)
    xb = (cent[rng.integers(0, 64, 20000)] + 0.5 * rng.standard_normal((20000, 256))).astype(np.float32)
    xb /= np.linalg.norm(xb, axis=1, keepdims=True)
    xq = (cent[rng.integers(0, 64, 200)] + 0.5 * rng.standard_normal((200, 256))).astype(np.float32)
    xq /= np.linalg.norm(xq, axis=1, keepdims=True)
    index = vf.IndexFlat(256, metric, dtype="bf16")
    index.add(xb)
    _, I = index.search(xq, 10)
    _, Ir = flat.knn_exact(xb, xq, 10, metric)
    recall = np.mean([len(set(I[q]) & set(Ir[q])) / 10 for q in range(200)])
    assert recall >= 0.9, recall


def test_bf16_selfjoin(vf):
    x = _rand(700, 48, 8)
    index = vf.IndexFlatIP(48, dtype="bf16")
    index.add(x)
    S, I = index.selfjoin(15)
    Sr, Ir = flat.pgvector_cosine_topk(flat.round_bf16(x), 15)
    diff = I != Ir
    for q, j in zip(*np.nonzero(diff)):
        assert abs(float(Sr[q, j]) - float(S[q, j])) < 1e-5
    np.testing.assert_allclose(S[~diff], Sr[~diff], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("metric", [L2, IP])
def test_bf16_tombstoned_removals(vf, metric, monkeypatch):
    """remove_ids on an index without filter planes (bf16 storage) tombstones
    the rows (NaN-filled in place, vs_api.hip vs_remove_ids) until the dead
    fraction reaches 1 / VS_PACK_DEN: faiss's labels (positions among the live
    rows) must come out of every search path — the small-batch kernels, the
    bf16 GEMM, the two-page k > 32 engine, raw lists — and out of reconstruct;
    appends continue the label space; a large removal packs; the self-join
    packs first.  Oracle: the fp64 search over the bf16-rounded live rows."""
    monkeypatch.setenv("VS_PACK_DEN", "16")
    d = 96
    xb = _rand(8000, d, 11)
    index = vf.IndexFlat(d, metric, dtype="bf16")
    index.add(xb)
    xr = flat.round_bf16(xb)
    rng = np.random.default_rng(12)

    def check(nq, k, seed, raw=False):
        xq = _rand(nq, d, seed)
        rq = flat.round_bf16(xq)
        D, I = index.search(xq, k, raw=raw)
        if raw:
            Dr, Ir = flat.knn_lex(xr, rq, k, metric)
        else:
            Dr, Ir = flat.knn_exact(xr, rq, k, metric)
        bad = flat.mismatches(D, I, Dr, Ir, metric, xr, rq)
        assert not bad, (nq, k, raw, bad[:3])

    for r in range(4):
        rm = rng.choice(xr.shape[0], 60, replace=False)  # well under 1/16: tombstones
        assert index.remove_ids(np.concatenate([rm, rm[:3], [10 ** 9]])) == 60
        xr, _ = flat.remove_ids(xr, rm)
        add = _rand(50, d, 20 + r)
        index.add(add)
        xr = np.concatenate([xr, flat.round_bf16(add)])
        assert index.ntotal == xr.shape[0]
        for nq in (1, 8, 40):
            check(nq, 10, 30 + r)
        for lab in rng.choice(xr.shape[0], 5, replace=False):
            np.testing.assert_array_equal(index.reconstruct(int(lab)), xr[lab])
        np.testing.assert_array_equal(index.reconstruct_n(0, index.ntotal), xr)
    if metric == IP:
        check(40, 50, 40)              # faiss's rule past k = 32 (two pages)
        check(40, 100, 41, raw=True)   # a shard's raw half of a sharded k = 50
    # a removal past 1/16 of the rows packs the tombstones (labels unchanged)
    rm = np.arange(0, xr.shape[0], 5, dtype=np.int64)
    assert index.remove_ids(rm) == rm.size
    xr, _ = flat.remove_ids(xr, rm)
    assert index.ntotal == xr.shape[0]
    check(40, 10, 50)
    np.testing.assert_array_equal(index.reconstruct_n(0, index.ntotal), xr)
    # tombstones again, then the self-join (which packs them first)
    rm = rng.choice(xr.shape[0], 40, replace=False)
    index.remove_ids(rm)
    xr, _ = flat.remove_ids(xr, rm)
    S, I = index.selfjoin(10)
    Sr, Ir = flat.pgvector_cosine_topk(xr, 10)
    diff = I != Ir
    for q, j in zip(*np.nonzero(diff)):
        assert abs(float(Sr[q, j]) - float(S[q, j])) < 1e-5
    assert index.ntotal == xr.shape[0]


def test_bf16_int8_plane_small_batches(vf, monkeypatch):
    """C5's path at reduced size: a bf16 inner-product index of 300,000 rows
    keeps an int8 plane; batches of up to 32 queries run the small-batch filter
    pass over it (1 B per element instead of the rows' 2) and the verification
    rescores the stored bf16 values in fp64, so the answers are the exact
    roundings (strict window) of the bf16 rows' scores.  Removals tombstone the
    rows (their plane factors become NaN and never enter a list), appends
    extend the plane, a large removal packs rows and plane together."""
    from vsearch import _lib

    monkeypatch.setenv("VS_PACK_DEN", "16")
    d, n = 128, 300_000
    rng = np.random.default_rng(21)
    xb = rng.standard_normal((n, d)).astype(np.float32)
    index = vf.IndexFlat(d, IP, dtype="bf16")
    index.add(xb)
    assert index.filter_planes == ("i8",)
    xr = flat.round_bf16(xb)

    def check(seed):
        for nq in (1, 8, 32):
            xq = _rand(nq, d, seed + nq)
            rq = flat.round_bf16(xq)
            _lib.filter_stats(reset=True)
            D, I = index.search(xq, 10)
            fq, _ = _lib.filter_stats(reset=True)
            assert fq == nq, (nq, fq)  # the int8 plane's filter pass ran
            Dr, Ir = flat.knn_exact(xr, rq, 10, IP)
            bad = flat.mismatches(D, I, Dr, Ir, IP, xr, rq, strict=True)
            assert not bad, (nq, bad[:3])

    check(100)
    for r in range(2):
        rm = rng.choice(xr.shape[0], 3000, replace=False)  # tombstones (1 %)
        assert index.remove_ids(rm) == 3000
        xr, _ = flat.remove_ids(xr, rm)
        add = _rand(2000, d, 200 + r)
        index.add(add)
        xr = np.concatenate([xr, flat.round_bf16(add)])
        assert index.ntotal == xr.shape[0]
        check(300 + r)
    rm = np.arange(0, xr.shape[0], 9, dtype=np.int64)  # past 1/16: packs
    assert index.remove_ids(rm) == rm.size
    xr, _ = flat.remove_ids(xr, rm)
    check(400)
    np.testing.assert_array_equal(index.reconstruct_n(0, 1000), xr[:1000])
