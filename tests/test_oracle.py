"""CPU: the oracle pinned against the reference's fixtures and its own restatements.

* the C faiss-heap restatement (oracle/faiss_flat.c) and the numpy rule agree on
  tie-heavy data (the only place the two could diverge);
* hand-derived known answers for the reference's 3-d embedding stub
  ([i%3]*3, query [0,0,0]: tests/test_integration_ingestion_graph.py:40-48);
* the committed golden vectors (tests/golden/) reproduce from the committed inputs;
* remove_ids / pgvector self-join / padding semantics.
"""

import numpy as np
import pytest

from oracle import cfaiss, flat

L2, IP = flat.METRIC_L2, flat.METRIC_INNER_PRODUCT


@pytest.mark.parametrize("metric", [L2, IP])
def test_c_heap_equals_numpy_rule(metric):
    rng = np.random.default_rng(0)
    for _ in range(300):
        n = int(rng.integers(1, 80))
        nq = int(rng.integers(1, 4))
        d = int(rng.integers(1, 4))
        k = int(rng.integers(1, 14))
        xb = rng.integers(-2, 3, size=(n, d)).astype(np.float32)
        xq = rng.integers(-2, 3, size=(nq, d)).astype(np.float32)
        Dc, Ic = cfaiss.knn_seq(xb, xq, k, metric)
        Dn, In = flat.knn_exact(xb, xq, k, metric)
        np.testing.assert_array_equal(Ic, In)
        np.testing.assert_array_equal(Dc, Dn)


def test_heap_select_on_scores_matches_rule():
    rng = np.random.default_rng(1)
    s = rng.integers(0, 4, size=(50, 40)).astype(np.float32)
    for metric in (L2, IP):
        for k in (1, 3, 7, 40, 45):
            Dc, Ic = cfaiss.heap_select(s, k, metric)
            Dn, In = flat.select_topk(s.astype(np.float64), k, metric)
            np.testing.assert_array_equal(Ic, In)


def test_reference_tie_stub_known_answers(golden):
    """Hand-derived from faiss's heaps: L2 keeps the lowest labels ascending; IP's
    CMin heap keeps labels 0..k-1 (strict admission, every score 0) and
    heap_reorder emits them in descending label order."""
    _, exp = golden
    xb = np.array([[float(i % 3)] * 3 for i in range(341)], dtype=np.float32)
    xq = np.zeros((1, 3), dtype=np.float32)
    for k in (1, 4, 5, 10):
        D, I = flat.knn_exact(xb, xq, k, L2)
        assert I[0].tolist() == [3 * j for j in range(k)]
        assert (D == 0).all()
        D, I = flat.knn_exact(xb, xq, k, IP)
        assert I[0].tolist() == list(range(k - 1, -1, -1))
        assert (D == 0).all()
        for m, name in ((L2, "l2"), (IP, "ip")):
            D, I = flat.knn_exact(xb, xq, k, m)
            np.testing.assert_array_equal(I, exp[f"tie_{name}_k{k}_I"])


def test_small_ip_tie_walkthrough():
    """faiss CMin heap, k=2, scores (id: 5, 5, 7): the later 7 evicts the top,
    which is the SMALLER label among the tied 5s -> result [2, 1]."""
    xb = np.array([[5.0], [5.0], [7.0]], dtype=np.float32)
    xq = np.ones((1, 1), dtype=np.float32)
    D, I = cfaiss.knn_seq(xb, xq, 2, IP)
    assert I[0].tolist() == [2, 1]
    D, I = flat.knn_exact(xb, xq, 2, IP)
    assert I[0].tolist() == [2, 1]
    # L2's CMax heap on the mirrored case keeps the LOWER tied label: dists 4, 4, 0
    xb2 = np.array([[2.0], [2.0], [0.0]], dtype=np.float32)
    xq2 = np.zeros((1, 1), dtype=np.float32)
    assert cfaiss.knn_seq(xb2, xq2, 2, L2)[1][0].tolist() == [2, 0]
    assert flat.knn_exact(xb2, xq2, 2, L2)[1][0].tolist() == [2, 0]


@pytest.mark.parametrize("metric", [L2, IP])
def test_golden_books_reproduce(golden, golden_vectors, metric):
    _, exp = golden
    xb, xq, _ = golden_vectors
    name = "l2" if metric == L2 else "ip"
    D, I = flat.knn_exact(xb, xq, 30, metric)
    np.testing.assert_array_equal(I, exp[f"books_{name}_I"])
    np.testing.assert_allclose(D, exp[f"books_{name}_D"], rtol=1e-6, atol=1e-6)
    if metric == L2:
        # every book is its own nearest neighbour at distance ~0
        assert (I[:341, 0] == np.arange(341)).all()


def test_golden_students_reproduce(golden, golden_vectors):
    _, exp = golden
    _, _, xs = golden_vectors
    for k in (15, 50):
        S, I = flat.pgvector_cosine_topk(xs, k)
        np.testing.assert_array_equal(I, exp[f"students_k{k}_I"])
        assert not (I == np.arange(25)[:, None]).any()
        # k > N - 1: 24 neighbours, then padding
        if k == 50:
            assert (I[:, 24:] == -1).all() and (I[:, :24] >= 0).all()


def test_golden_inputs_consistent(golden):
    inputs, _ = golden
    assert len(inputs["book_texts"]) == 341
    assert len(inputs["book_metadata"]) == 341
    assert len(inputs["student_keys"]) == 25
    assert inputs["book_metadata"][0]["book_id"] == "B001"
    assert inputs["book_texts"][0].startswith("Charlotte's Web by E.B. White. Genre: fiction, classic.")


def test_padding_and_empty():
    xb = np.eye(3, dtype=np.float32)
    for metric in (L2, IP):
        D, I = flat.knn_exact(xb, np.ones((2, 3), np.float32), 5, metric)
        assert (I[:, 3:] == -1).all()
        assert (D[:, 3:] == flat.neutral(metric)).all()
        D, I = flat.knn_exact(np.zeros((0, 3), np.float32), np.ones((1, 3), np.float32), 2, metric)
        assert (I == -1).all()
    assert flat.neutral(L2) == np.finfo(np.float32).max


def test_nan_and_neutral_never_admitted():
    s = np.array([[np.nan, 1.0, np.finfo(np.float32).max, 0.5]], dtype=np.float64)
    D, I = flat.select_topk(s, 4, L2)
    assert I[0].tolist() == [3, 1, -1, -1]
    D, I = flat.select_topk(-s, 4, IP)
    assert I[0].tolist() == [3, 1, -1, -1]


def test_remove_ids_semantics():
    xb = np.arange(20, dtype=np.float32).reshape(10, 2)
    xr, n = flat.remove_ids(xb, [3, 3, 0, 99, -1, 9])
    assert n == 3
    np.testing.assert_array_equal(xr[:, 0], [2, 4, 8, 10, 12, 14, 16])


def test_pgvector_selfjoin_semantics():
    x = np.array([[1, 0], [1, 0.1], [0, 1], [0, 0], [1, 0]], dtype=np.float32)
    S, I = flat.pgvector_cosine_topk(x, 4)
    # row 0: row 4 identical (sim 1), then row 1; zero row 3 never appears
    assert I[0, 0] == 4 and I[0, 1] == 1
    assert not (I == 3).any()
    assert (I[3] == -1).all()
    S2, I2 = flat.pgvector_cosine_topk(x, 4, min_sim=0.75)
    assert set(I2[0][I2[0] >= 0].tolist()) == {4, 1}


@pytest.mark.parametrize("metric", [L2, IP])
def test_fp32_baseline_port_agrees(metric):
    rng = np.random.default_rng(3)
    xb = rng.standard_normal((5000, 64)).astype(np.float32)
    xq = rng.standard_normal((30, 64)).astype(np.float32)
    D, I = flat.knn_faiss_fp32(xb, xq, 10, metric, bs_y=1024)
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xb, xq)


def test_mismatch_checker_catches_errors():
    rng = np.random.default_rng(4)
    xb = rng.standard_normal((200, 8)).astype(np.float32)
    xq = rng.standard_normal((3, 8)).astype(np.float32)
    D, I = flat.knn_exact(xb, xq, 5, L2)
    I2 = I.copy()
    I2[0, 2] = I[0, 4]
    I2[0, 4] = I[0, 2]
    assert flat.mismatches(D, I2, D, I, L2, xb, xq)
    D2 = D.copy()
    D2[1, 1] += 0.01
    assert flat.mismatches(D2, I, D, I, L2, xb, xq)


@pytest.mark.parametrize("metric", [L2, IP])
def test_vectorised_checker_agrees_with_mismatches(metric):
    """mismatches_vec (the large-k checker of tests/test_gpu_wide_k.py) accepts
    what mismatches accepts and catches what it catches: the fp32 results
    themselves, swapped labels, off scores, padding and duplicates; and the C
    heap agrees with the numpy rule past one 64-entry page (k up to 300)."""
    rng = np.random.default_rng(5)
    xb = rng.standard_normal((400, 8)).astype(np.float32)
    xq = rng.standard_normal((20, 8)).astype(np.float32)
    for k in (5, 100, 450):
        Dr, Ir = flat.knn_exact(xb, xq, k, metric)
        Df, If = flat.knn_faiss_fp32(xb, xq, k, metric)
        assert not flat.mismatches_vec(Df, If, Dr, Ir, metric, xb, xq)
        assert not flat.mismatches(Df, If, Dr, Ir, metric, xb, xq)
        I2 = Ir.copy()
        I2[3, [1, 4]] = Ir[3, [4, 1]]
        assert flat.mismatches_vec(Dr, I2, Dr, Ir, metric, xb, xq)
        D2 = Dr.copy()
        D2[7, 2] += 0.01
        assert flat.mismatches_vec(D2, Ir, Dr, Ir, metric, xb, xq)
        I3 = Ir.copy()
        I3[0, 1] = Ir[0, 0]
        assert flat.mismatches_vec(Dr, I3, Dr, Ir, metric, xb, xq)
    xi = rng.integers(-2, 3, size=(600, 3)).astype(np.float32)
    qi = rng.integers(-2, 3, size=(4, 3)).astype(np.float32)
    for k in (65, 100, 300):
        Dc, Ic = cfaiss.knn_seq(xi, qi, k, metric)
        Dn, In = flat.knn_exact(xi, qi, k, metric)
        np.testing.assert_array_equal(Ic, In)
        np.testing.assert_array_equal(Dc, Dn)


def _engine_keys(xb, xq, metric):
    """The filter engine's final keys restated in numpy: fp64 dot products
    rounded once, fp64-summed norms rounded once, L2 by faiss's BLAS formula in
    fp32 (vs_gemm_x1.hip exact_key, vs_device.h l2_from_ip)."""
    ip = (xq.astype(np.float64) @ xb.astype(np.float64).T).astype(np.float32)
    if metric == IP:
        return ip
    qn = np.einsum("ij,ij->i", xq.astype(np.float64), xq.astype(np.float64)).astype(np.float32)
    xn = np.einsum("ij,ij->i", xb.astype(np.float64), xb.astype(np.float64)).astype(np.float32)
    return np.maximum((qn[:, None] + xn[None, :]) - np.float32(2) * ip, np.float32(0))


@pytest.mark.parametrize("metric", [L2, IP])
def test_strict_checker_accepts_rounded_keys_and_rejects_near_swaps(metric):
    """strict=True accepts exactly what an exactly rescored engine can return
    (its keys within key_window of the fp64 score, labels swapped only inside
    overlapping windows) and rejects a near-neighbour swap that the fp32
    contract's 1e-5 window would let through."""
    rng = np.random.default_rng(5)
    xb = rng.standard_normal((3000, 1536)).astype(np.float32)
    xq = rng.standard_normal((8, 1536)).astype(np.float32)
    keys = _engine_keys(xb, xq, metric)
    D, I = flat.select_topk(keys.astype(np.float64), 10, metric, rule="lex")
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
    # a near-duplicate of query 0's best row, slightly worse: its exact score is
    # inside 1e-5 relative but far outside the rounding window
    best = int(Ir[0, 0])
    s0 = flat.exact_scores(xb[best:best + 1], xq[:1], metric)[0, 0]
    eps = 3e-6 * max(abs(s0), 1.0)
    step = xq[0] / np.linalg.norm(xq[0])
    xb2 = np.concatenate([xb, (xb[best] - (eps / np.linalg.norm(xq[0])) * step)[None]]).astype(np.float32)
    new = xb2.shape[0] - 1
    Dr2, Ir2 = flat.knn_exact(xb2, xq, 10, metric)
    assert Ir2[0, 1] == new  # the oracle ranks it second
    I_sw = Ir2.copy()
    I_sw[0, 0], I_sw[0, 1] = Ir2[0, 1], Ir2[0, 0]
    D_sw = Dr2.copy()
    D_sw[0, 0], D_sw[0, 1] = Dr2[0, 1], Dr2[0, 0]
    assert flat.mismatches(D_sw, I_sw, Dr2, Ir2, metric, xb2, xq, strict=True)
    if metric == IP:  # the old 1e-5 window would have accepted the swap
        assert not [b for b in flat.mismatches(D_sw, I_sw, Dr2, Ir2, metric, xb2, xq)
                    if b[2] == "label"]
    # a score that is not the rounding of the label's exact score
    D_off = D.copy()
    D_off[1, 3] = np.nextafter(np.nextafter(D[1, 3], np.inf, dtype=np.float32), np.inf,
                               dtype=np.float32) if metric == IP else D[1, 3] * np.float32(1 + 1e-5)
    assert flat.mismatches(D_off, I, Dr, Ir, metric, xb, xq, strict=True)


def test_strict_selfjoin_checker():
    rng = np.random.default_rng(6)
    x = rng.standard_normal((400, 64)).astype(np.float32)
    Sr, Ir = flat.pgvector_cosine_topk(x, 10)
    assert not flat.selfjoin_mismatches(Sr, Ir, Sr, Ir, x, np.arange(400), strict=True)
    S2 = Sr.copy()
    S2[3, 2] += 2e-6
    assert flat.selfjoin_mismatches(S2, Ir, Sr, Ir, x, np.arange(400), strict=True)
    assert not flat.selfjoin_mismatches(S2, Ir, Sr, Ir, x, np.arange(400))


@pytest.mark.parametrize("metric", [IP, L2])
def test_simd_speed_standin_matches_scalar_labels(metric):
    """oracle/faiss_flat_simd.c (the faiss-speed stand-in bench.py times for
    nq = 1) scans the same rows with reassociated sums: on separated float
    data its labels equal the scalar heap oracle's and its scores agree to
    fp32 rounding."""
    rng = np.random.default_rng(17)
    xb = rng.standard_normal((3000, 100)).astype(np.float32)
    xq = rng.standard_normal((3, 100)).astype(np.float32)
    D, I = cfaiss.knn_seq(xb, xq, 10, metric)
    Ds, Is = cfaiss.knn_seq_simd(xb, xq, 10, metric)
    np.testing.assert_array_equal(Is, I)
    np.testing.assert_allclose(Ds, D, rtol=1e-5, atol=1e-4)
