"""GPU parity: libvsearch.so (HIP, gfx950) against the CPU oracle.

Every test here runs the product path through the C-ABI on cuda:0 and checks it
with oracle/flat.py (fp64 semantics of faiss IndexFlat::search) or the C heap
restatement oracle/faiss_flat.c.  Acceptance (oracle.flat.mismatches):
* searches the staged filter-and-verify engine answers (fp32 rows, more than
  32 queries, IP k <= 28 / L2 k <= 56; _staged) are checked STRICTLY: every D is
  the fp32 rounding of its label's fp64 score (flat.key_window) and a label
  differs from the oracle's only inside a true fp32-key tie;
* the fp32-accumulating engines (GEMV, skinny, the fp32 MFMA GEMM: faiss's own
  arithmetic class) meet the north star's fp32 contract: labels equal except
  ties within, and scores within, 1e-5 * max(1, |s|) (for squared L2 the scale
  includes |q|^2 + |x|^2, the magnitude fp32 rounding acts on)."""

import numpy as np
import pytest

from helpers import assert_against_candidates
from oracle import cfaiss, flat

pytestmark = pytest.mark.gpu

L2, IP = flat.METRIC_L2, flat.METRIC_INNER_PRODUCT


@pytest.fixture(scope="module")
def vf():
    from vsearch import _lib
    from vsearch import faiss as vfaiss

    assert _lib.device_count() >= 1, "gpu tests need a visible MI355X"
    return vfaiss


# Filter-and-verify planes: int8 (the first stage by default) and bf16; an L2
# index's int8 plane holds the augmented rows (L2 as an inner product,
# vs_gemm_x1.hip quantize_i8_l2aug_kernel).
FILTER_CASES = [(L2, "bf16v"), (L2, "i8v"), (IP, "bf16v"), (IP, "i8v")]


def _rand(n, d, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        return rng.standard_normal((n, d)).astype(np.float32)
    if kind == "int":
        return rng.integers(-2, 3, size=(n, d)).astype(np.float32)
    raise ValueError(kind)


def _staged(metric, nq, k, engine="auto"):
    """Whether a search of an fp32 index is answered by the staged
    filter-and-verify engine (vs_api.hip run_topk: more than kSkinnyMaxQ = 32
    queries and a candidate count x1_list_len(need) > 0, need = 2k - 1 for IP)."""
    need = 2 * k - 1 if metric == IP else k
    return engine != "fp32" and nq > 32 and need + 8 <= 64


def _check(vf, xb, xq, k, metric):
    index = vf.IndexFlat(xb.shape[1], metric)
    index.add(xb)
    D, I = index.search(xq, k)
    Dr, Ir = flat.knn_exact(xb, xq, k, metric)
    strict = _staged(metric, xq.shape[0], k) and xb.shape[0] > 0
    bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=strict)
    assert not bad, (strict, bad[:5])
    return D, I


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("nq", [1, 2, 3, 5, 8, 9, 20, 37, 129])
def test_shapes_nq(vf, metric, nq):
    xb = _rand(3000, 96, 1)
    xq = _rand(nq, 96, 2)
    _check(vf, xb, xq, 10, metric)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("k", [1, 2, 4, 5, 8, 9, 16, 17, 20, 30, 33, 50, 64])
def test_k_values(vf, metric, k):
    xb = _rand(2000, 64, 3)
    for nq in (1, 40):
        _check(vf, xb, _rand(nq, 64, 4 + nq), k, metric)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("n", [1, 2, 7, 127, 128, 129, 255, 256, 257, 1000])
def test_ragged_ntotal(vf, metric, n):
    xb = _rand(n, 40, 5)
    for nq in (1, 4, 33):
        _check(vf, xb, _rand(nq, 40, 6), 10, metric)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("d", [1, 3, 31, 32, 33, 100, 768, 1536, 2049])
def test_dims(vf, metric, d):
    xb = _rand(700, d, 7)
    for nq in (1, 3, 25):
        _check(vf, xb, _rand(nq, d, 8), 5, metric)


@pytest.mark.parametrize("metric", [L2, IP])
def test_k_exceeds_ntotal_padding(vf, metric):
    xb = _rand(5, 16, 9)
    for nq in (1, 30):
        D, I = _check(vf, xb, _rand(nq, 16, 10), 12, metric)
        assert (I[:, 5:] == -1).all()
        assert (D[:, 5:] == flat.neutral(metric)).all()


@pytest.mark.parametrize("metric", [L2, IP])
def test_empty_index(vf, metric):
    index = vf.IndexFlat(8, metric)
    D, I = index.search(_rand(3, 8, 11), 4)
    assert (I == -1).all() and (D == flat.neutral(metric)).all()
    D, I = index.search(np.zeros((0, 8), np.float32), 4)
    assert D.shape == (0, 4) and I.shape == (0, 4)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("k", [1, 2, 4, 5, 10, 16, 33, 50, 60, 64])
def test_ties_match_faiss_heap(vf, metric, k):
    """Tie-heavy integer data: labels must equal the C faiss-heap restatement
    exactly.  Inner product with k > 32 reads up to 2k - 1 = 127 entries: the
    two-page search (vs_api.hip run_wide_k; nq = 1 on the GEMV, 7 and 40 on the
    fp32 MFMA GEMM; service.py:529-531 asks for k = 60)."""
    xb = _rand(600, 3, 12, "int")
    for nq in (1, 7, 40):
        xq = _rand(nq, 3, 13 + nq, "int")
        index = vf.IndexFlat(3, metric)
        index.add(xb)
        D, I = index.search(xq, k)
        Dc, Ic = cfaiss.knn_seq(xb, xq, k, metric)
        np.testing.assert_array_equal(I, Ic)
        np.testing.assert_array_equal(D, Dc)


@pytest.mark.parametrize("nq", [1, 2, 5, 300])
@pytest.mark.parametrize("k", [40, 60, 64])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_ip_wide_k_duplicate_rows(vf, nq, k, dtype):
    """Float rows with a block of 150 duplicates (the re-ingested book of
    book_vector/main.py:148, which add_texts appends again): the duplicates'
    run of equal keys fills the first page, and faiss's rule picks the k
    smallest of their labels (descending); checked against the C heap
    restatement (labels exact, scores within the fp32 contract).  The bf16
    storage variant (C5) runs the same two pages on its own operands (qb16
    queries, 2-byte rows): the oracle sees the bf16-rounded rows and queries."""
    d = 64
    xb = _rand(6000, d, 71)
    dup = _rand(1, d, 72)[0]
    pos = np.random.default_rng(73).choice(6000, 150, replace=False)
    xb[pos] = dup
    xq = _rand(nq, d, 74) * 0.05 + dup  # near the duplicated row
    index = vf.IndexFlat(d, IP, dtype=dtype)
    index.add(xb)
    D, I = index.search(xq, k)
    if dtype == "bf16":
        xb, xq = flat.round_bf16(xb), flat.round_bf16(xq)
    Dc, Ic = cfaiss.knn_seq(xb, xq, k, IP)
    np.testing.assert_array_equal(I, Ic)
    np.testing.assert_allclose(D, Dc, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("nq", [1, 7, 200])
@pytest.mark.parametrize("k", [65, 100, 127])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_raw_search_beyond_64(vf, nq, k, dtype):
    """VS_RAW_ORDER inner-product searches of up to 2 * VS_MAX_K entries (a
    shard's half of a sharded k > 32 search): the lexicographic (key, label)
    order, both pages, against the fp64 oracle; integer rows (exact scores,
    also in bf16 storage: small integers are bf16 values)."""
    xb = _rand(900, 4, 81, "int")
    xq = _rand(nq, 4, 82, "int")
    index = vf.IndexFlat(4, IP, dtype=dtype)
    index.add(xb)
    D, I = index.search(xq, k, raw=True)
    Dr, Ir = flat.knn_lex(xb, xq, k, IP)
    np.testing.assert_array_equal(I, Ir)
    np.testing.assert_array_equal(D, Dr)


@pytest.mark.parametrize("metric", [L2, IP])
def test_reference_tie_stub(vf, metric, golden):
    """The reference's embedding stub [i%3]*3 with query [0,0,0]
    (tests/test_integration_ingestion_graph.py:40-48)."""
    _, exp = golden
    name = "l2" if metric == L2 else "ip"
    xb = np.array([[float(i % 3)] * 3 for i in range(341)], dtype=np.float32)
    index = vf.IndexFlat(3, metric)
    index.add(xb)
    for k in (1, 4, 5, 10):
        D, I = index.search(np.zeros((1, 3), np.float32), k)
        np.testing.assert_array_equal(I, exp[f"tie_{name}_k{k}_I"])
        np.testing.assert_array_equal(D, exp[f"tie_{name}_k{k}_D"])


@pytest.mark.parametrize("metric", [L2, IP])
def test_golden_csv_books(vf, metric, golden, golden_vectors):
    """BASELINE config 1: catalog_sample.csv books with deterministic embeddings."""
    _, exp = golden
    xb, xq, _ = golden_vectors
    name = "l2" if metric == L2 else "ip"
    index = vf.IndexFlat(xb.shape[1], metric)
    index.add(xb)
    for k in (4, 5, 10, 20, 30):
        for q in (xq[:1], xq[:7], xq):
            D, I = index.search(q, k)
            Ir = exp[f"books_{name}_I"][: q.shape[0], :k]
            Dr = exp[f"books_{name}_D"][: q.shape[0], :k]
            strict = _staged(metric, q.shape[0], k)
            bad = flat.mismatches(D, I, Dr, Ir, metric, xb, q, strict=strict)
            assert not bad, (strict, bad[:5])
            # fp32 vs fp64 near-ties may swap neighbours; they must stay rare
            assert (I != Ir).mean() < 1e-3


def test_golden_csv_students_selfjoin(vf, golden, golden_vectors):
    """graph_refresher self-join on students_sample.csv (k=15 and 50 > N-1)."""
    _, exp = golden
    _, _, xs = golden_vectors
    index = vf.IndexFlatIP(xs.shape[1])
    index.add(xs)
    for k in (15, 50):
        S, I = index.selfjoin(k)
        np.testing.assert_array_equal(I, exp[f"students_k{k}_I"])
        np.testing.assert_allclose(S, exp[f"students_k{k}_S"], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("k", [1, 5, 15, 50])
def test_selfjoin_random(vf, k):
    x = _rand(1500, 64, 14)
    x[17] = 0.0  # zero-norm row: never a neighbour, no neighbours (pgvector NaN)
    index = vf.IndexFlatL2(64)
    index.add(x)
    S, I = index.selfjoin(k)
    Sr, Ir = flat.pgvector_cosine_topk(x, k)
    assert (I[17] == -1).all()
    assert not (I == 17).any()
    assert not (I == np.arange(1500)[:, None]).any()
    # the staged engine (k <= 56): similarities are roundings of the exact
    # cosine, labels differ only inside a true tie (flat.key_window)
    bad = flat.selfjoin_mismatches(S, I, Sr, Ir, x, np.arange(1500), strict=k <= 56)
    assert not bad, bad[:5]


@pytest.mark.parametrize("engine", ["i8v", "bf16v"])
@pytest.mark.parametrize("k", [10, 50])
def test_selfjoin_filter_fallback_drops_self(vf, k, engine):
    """Cosine self-join through the filter engine with 40-fold duplicated rows: the
    tied candidates cannot be separated by the bound, those students are redone
    as plain searches for k + 1 and lose their own row; parity with the oracle."""
    from vsearch import _lib

    base = _rand(30, 96, 72)
    x = np.concatenate([np.repeat(base, 40, axis=0), _rand(600, 96, 73)])
    index = vf.IndexFlatIP(96)
    index.set_engine(engine)
    index.add(x)
    _lib.filter_stats(reset=True)
    S, I = index.selfjoin(k)
    nq, nfb = _lib.filter_stats(reset=True)
    assert nq == x.shape[0]
    if k == 10:  # 39 exact ties at similarity 1: every duplicated row falls back
        assert nfb >= 1000
    Sr, Ir = flat.pgvector_cosine_topk(x, k)
    assert not (I == np.arange(x.shape[0])[:, None]).any()
    # the redo stage rescores its candidates too: strict like every stage
    bad = flat.selfjoin_mismatches(S, I, Sr, Ir, x, np.arange(x.shape[0]), strict=True)
    assert not bad, bad[:5]


def test_selfjoin_threshold_and_subrange(vf):
    rng = np.random.default_rng(15)
    base = rng.standard_normal((40, 32)).astype(np.float32)
    x = np.concatenate([base, base + 0.1 * rng.standard_normal((40, 32)).astype(np.float32)])
    index = vf.IndexFlatIP(32)
    index.add(x)
    S, I = index.selfjoin(15, q0=10, nq=50, min_sim=0.75)
    Sr, Ir = flat.pgvector_cosine_topk(x, 15, q_rows=np.arange(10, 60), min_sim=0.75)
    np.testing.assert_array_equal(I, Ir)
    m = I >= 0
    np.testing.assert_allclose(S[m], Sr[m], rtol=1e-5, atol=1e-6)
    assert (S[~m] == -flat.FLT_MAX).all()


def test_add_incremental_reconstruct_remove(vf):
    xb = _rand(1000, 24, 16)
    index = vf.IndexFlatL2(24)
    for i0 in range(0, 1000, 137):
        index.add(xb[i0:i0 + 137])
    assert index.ntotal == 1000
    np.testing.assert_array_equal(index.reconstruct(0), xb[0])
    np.testing.assert_array_equal(index.reconstruct(999), xb[999])
    np.testing.assert_array_equal(index.reconstruct_n(100, 50), xb[100:150])
    with pytest.raises(RuntimeError):
        index.reconstruct(1000)
    rm = np.array([5, 0, 999, 5, 4000, -3, 500], dtype=np.int64)
    n = index.remove_ids(rm)
    xr, nr = flat.remove_ids(xb, rm)
    assert n == nr == 4
    assert index.ntotal == 996
    np.testing.assert_array_equal(index.reconstruct_n(0, 996), xr)
    xq = _rand(30, 24, 17)
    D, I = index.search(xq, 7)
    Dr, Ir = flat.knn_exact(xr, xq, 7, L2)
    assert not flat.mismatches(D, I, Dr, Ir, L2, xr, xq)
    index.add(xb[:10])
    assert index.ntotal == 1006
    index.reset()
    assert index.ntotal == 0


def test_remove_many_chunks(vf):
    """remove_ids across several compaction chunks (chunk = 256 MiB of rows)."""
    d = 1536
    n = 60000  # 368 MB -> two chunks
    index = vf.IndexFlatIP(d)
    index.add_synthetic(n, seed=77)
    rng = np.random.default_rng(18)
    rm = rng.choice(n, 3000, replace=False).astype(np.int64)
    assert index.remove_ids(rm) == 3000
    keep = np.setdiff1d(np.arange(n), rm)
    from vsearch.synth import synthetic_rows

    for r in (0, 1, 2, keep.size // 2, keep.size - 1):
        np.testing.assert_array_equal(index.reconstruct(r), synthetic_rows(keep[r], 1, d, 77)[0])


def test_remove_packs_in_place_once_the_shift_covers_a_chunk(vf):
    """The compaction's two forms (vs_remove_ids): a dense run of 24,000
    removed rows first (scratch chunk of 43,690 rows: the shift is smaller
    than the chunk), then every 9th row, moved straight to their final rows
    in chunks cut to the shift.  Every kept row, its norm (L2 keys) and the
    int8 plane (re-derived from the moved rows) are checked."""
    d, n = 1536, 120_000
    rng = np.random.default_rng(41)
    xb = rng.standard_normal((n, d), dtype=np.float32)
    index = vf.IndexFlatL2(d)
    index.add(xb)
    rm = np.concatenate([np.arange(500, 24_500), np.arange(24_500, n, 9)]).astype(np.int64)
    assert index.remove_ids(rm[::-1].copy()) == rm.size
    xr, nr = flat.remove_ids(xb, rm)
    assert nr == rm.size and index.ntotal == n - rm.size
    np.testing.assert_array_equal(index.reconstruct_n(0, index.ntotal), xr)
    xq = rng.standard_normal((16, d), dtype=np.float32)
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xr, xq, 10, L2)
    assert not flat.mismatches(D, I, Dr, Ir, L2, xr, xq)
    ip = vf.IndexFlatIP(d)
    ip.add(xb)
    ip.remove_ids(rm)
    D, I = ip.search(xq, 10)  # the filter engine on the re-derived int8 plane
    Dr, Ir = flat.knn_exact(xr, xq, 10, flat.METRIC_INNER_PRODUCT)
    assert not flat.mismatches(D, I, Dr, Ir, flat.METRIC_INNER_PRODUCT, xr, xq)


def test_synthetic_generator_matches_host(vf):
    from vsearch.synth import synthetic_rows

    index = vf.IndexFlatL2(1536)
    index.add_synthetic(300, seed=1234, row0=9_999_800)
    np.testing.assert_array_equal(index.reconstruct_n(0, 300),
                                  synthetic_rows(9_999_800, 300, 1536, 1234))


def test_device_pointer_search(vf):
    torch = pytest.importorskip("torch")
    xb = _rand(5000, 128, 19)
    xq = _rand(64, 128, 20)
    index = vf.IndexFlatIP(128)
    index.add(xb)
    q = torch.from_numpy(xq).cuda()
    D = torch.empty((64, 10), dtype=torch.float32, device="cuda")
    I = torch.empty((64, 10), dtype=torch.int64, device="cuda")
    index.search_device(q.data_ptr(), 64, 10, D.data_ptr(), I.data_ptr(),
                        torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    Dh, Ih = index.search(xq, 10)
    np.testing.assert_array_equal(I.cpu().numpy(), Ih)
    np.testing.assert_array_equal(D.cpu().numpy(), Dh)


@pytest.mark.parametrize("metric", [L2, IP])
def test_merge_topk_kernel(vf, metric):
    """vs_merge_topk (the post-all-gather merge) equals one index over all rows."""
    torch = pytest.importorskip("torch")
    import ctypes

    from vsearch import _lib

    xb = _rand(4000, 32, 21)
    xq = _rand(50, 32, 22)
    k = 10
    parts = []
    for lo, hi in ((0, 1000), (1000, 2500), (2500, 4000)):
        idx = vf.IndexFlat(32, metric)
        idx.add(xb[lo:hi])
        idx.set_id_base(lo)
        parts.append(idx.search(xq, k))
    Dp = torch.from_numpy(np.stack([p[0] for p in parts])).cuda()
    Ip = torch.from_numpy(np.stack([p[1] for p in parts])).cuda()
    D = torch.empty((50, k), dtype=torch.float32, device="cuda")
    I = torch.empty((50, k), dtype=torch.int64, device="cuda")
    _lib.check(_lib.load().vs_merge_topk(
        ctypes.c_void_p(Dp.data_ptr()), ctypes.c_void_p(Ip.data_ptr()), 3, 50, k, k, metric,
        ctypes.c_void_p(D.data_ptr()), ctypes.c_void_p(I.data_ptr()), None))
    torch.cuda.synchronize()
    Dr, Ir = flat.knn_exact(xb, xq, k, metric)
    bad = flat.mismatches(D.cpu().numpy(), I.cpu().numpy(), Dr, Ir, metric, xb, xq)
    assert not bad, bad[:5]


def test_errors(vf):
    index = vf.IndexFlatL2(16)
    index.add(_rand(10, 16, 23))
    with pytest.raises(AssertionError):
        index.search(_rand(2, 15, 24), 3)
    with pytest.raises(AssertionError):
        index.search(_rand(2, 16, 24), 0)
    with pytest.raises(AssertionError):
        index.add(_rand(2, 17, 24))
    D, I = index.search(_rand(2, 16, 24), 65)  # any k, as faiss-cpu: padded past ntotal
    assert (I[:, 10:] == -1).all() and sorted(I[0, :10]) == list(range(10))


@pytest.mark.parametrize("metric", [L2, IP])
def test_large_synthetic_sampled(vf, metric):
    """1M x 1536 (BASELINE config 2 shape, B=1024) checked on a query sample."""
    from vsearch.synth import synthetic_rows

    n, d, k = 1_000_000, 1536, 10
    index = vf.IndexFlat(d, metric)
    index.reserve(n)
    index.add_synthetic(n, seed=1234)
    xq = synthetic_rows(50_000_000, 1024, d, 5678)
    D, I = index.search(xq, k)
    # property checks on every query: sorted, unique, in range
    assert (I >= 0).all() and (I < n).all()
    if metric == L2:
        assert (np.diff(D, axis=1) >= 0).all()
    else:
        assert (np.diff(D, axis=1) <= 0).all()
    # exact check on a sample of queries against a chunked fp64 oracle: the 64
    # best rows by exact score with their norms, then the strict check (the
    # staged engine answers B = 1024)
    sample = [0, 1, 511, 1023]
    m = 64
    best_k = np.zeros((len(sample), 0))
    best_i = np.zeros((len(sample), 0), np.int64)
    best_n = np.zeros((len(sample), 0))
    step = 100_000
    for r0 in range(0, n, step):
        xb = synthetic_rows(r0, step, d, 1234)
        s = flat.exact_scores(xb, xq[sample], metric)
        key = s if metric == L2 else -s
        xn2 = np.einsum("ij,ij->i", xb.astype(np.float64), xb.astype(np.float64))
        best_k = np.concatenate([best_k, key], axis=1)
        best_i = np.concatenate([best_i, np.broadcast_to(np.arange(r0, r0 + step), key.shape)], axis=1)
        best_n = np.concatenate([best_n, np.broadcast_to(xn2, key.shape)], axis=1)
        part = np.argpartition(best_k, m - 1, axis=1)[:, :m]
        best_k = np.take_along_axis(best_k, part, axis=1)
        best_i = np.take_along_axis(best_i, part, axis=1)
        best_n = np.take_along_axis(best_n, part, axis=1)
    for row, q in enumerate(sample):
        exact = best_k[row] if metric == L2 else -best_k[row]
        qn2 = float(np.dot(xq[q].astype(np.float64), xq[q].astype(np.float64)))
        assert_against_candidates(D[q], I[q], (best_i[row], exact, best_n[row], qn2), metric, k, d,
                                  strict=True)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("nq", [1, 2, 5, 8, 13, 16, 17, 24, 32, 33])
def test_small_batch_paths(vf, metric, nq):
    """nq <= 32 runs the skinny MFMA kernel (fp32 L2 with nq <= 8: the GEMV)."""
    xb = _rand(5000, 128, 30)
    xq = _rand(nq, 128, 31)
    for k in (1, 10, 16, 30):
        _check(vf, xb, xq, k, metric)


@pytest.mark.parametrize("metric", [L2, IP])
def test_small_batch_ragged_rows(vf, metric):
    for n in (1, 63, 64, 65, 255, 256, 257, 4097):
        xb = _rand(n, 64, 32)
        for nq in (3, 20):
            _check(vf, xb, _rand(nq, 64, 33), 8, metric)


@pytest.mark.parametrize("metric,engine", [(L2, "fp32"), (IP, "fp32")] + FILTER_CASES)
def test_large_batch_engines(vf, engine, metric):
    """Every large-batch engine of fp32 indexes meets the fp32 tolerance."""
    xb = _rand(9000, 1536, 40) * 0.05
    xq = _rand(300, 1536, 41) * 0.05
    index = vf.IndexFlat(1536, metric)
    index.set_engine(engine)
    index.add(xb)
    for k in (1, 10, 32):
        D, I = index.search(xq, k)
        Dr, Ir = flat.knn_exact(xb, xq, k, metric)
        strict = _staged(metric, xq.shape[0], k, engine)  # IP k = 32: the fp32 engine
        bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=strict)
        assert not bad, (engine, k, strict, bad[:5])


@pytest.mark.parametrize("metric,engine", FILTER_CASES)
@pytest.mark.parametrize("d", [64, 128, 192, 96, 160, 1536])
def test_filter_step_shapes(vf, metric, engine, d):
    """The filter pass walks K in 64-element steps of the zero-padded rows (d = 96
    and 160 pad to 128 and 192); several tiles, a ragged last tile and a ragged
    query tile."""
    xb = _rand(1800, d, 46)
    xq = _rand(300, d, 47)
    index = vf.IndexFlat(d, metric)
    index.set_engine(engine)
    index.add(xb)
    for k in (1, 10):
        D, I = index.search(xq, k)
        Dr, Ir = flat.knn_exact(xb, xq, k, metric)
        bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
        assert not bad, (d, k, bad[:5])


@pytest.mark.parametrize("metric,engine", [(IP, "i8v"), (IP, "bf16v"), (L2, "i8v")])
def test_filter_plane_follows_mutations(vf, metric, engine):
    """The filter plane (codes, scales) and residual norms follow add /
    remove_ids / reset / storage growth (kept in step with the rows, never
    rebuilt lazily); for L2 the augmented plane's norms |x'|^2 too, with the
    augmentation fixed by the first add (later rows of larger norm than the
    first ones included)."""
    xb = _rand(3000, 96, 42)
    xb[2500:] *= 3.0  # larger rows after the augmentation is fixed
    xq = _rand(150, 96, 43)
    index = vf.IndexFlat(96, metric)
    index.set_engine(engine)
    index.add(xb[:2000])
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xb[:2000], xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xb[:2000], xq, strict=True)
    for i0 in range(2000, 3000, 250):  # several growths
        index.add(xb[i0:i0 + 250])
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
    rm = np.arange(100, 3000, 3, dtype=np.int64)
    index.remove_ids(rm)
    xr, _ = flat.remove_ids(xb, rm)
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xr, xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xr, xq, strict=True)
    index.reset()
    index.add(xb[:50])
    D, I = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xb[:50], xq, 10, metric)
    assert not flat.mismatches(D, I, Dr, Ir, metric, xb[:50], xq, strict=True)


@pytest.mark.parametrize("engine", ["fp32", "bf16v", "i8v"])
def test_selfjoin_engines(vf, engine):
    x = _rand(2000, 256, 44)
    index = vf.IndexFlatIP(256)
    index.set_engine(engine)
    index.add(x)
    S, I = index.selfjoin(15)
    Sr, Ir = flat.pgvector_cosine_topk(x, 15)
    bad = flat.selfjoin_mismatches(S, I, Sr, Ir, x, np.arange(2000), strict=engine != "fp32")
    assert not bad, (engine, bad[:5])


@pytest.mark.parametrize("metric,engine", FILTER_CASES)
def test_filter_ragged_shapes(vf, metric, engine):
    """Odd d (column padding), ragged row tiles, several query tiles per split,
    fewer rows than one tile."""
    for n, d, nq in ((5000, 100, 1000), (257, 1536, 129), (70001, 32, 256), (40, 64, 300)):
        xb = _rand(n, d, 45)
        xq = _rand(nq, d, 46)
        index = vf.IndexFlat(d, metric)
        index.set_engine(engine)
        index.add(xb)
        for k in (5, 10):
            D, I = index.search(xq, k)
            Dr, Ir = flat.knn_exact(xb, xq, k, metric)
            bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
            assert not bad, (n, d, nq, k, bad[:5])


@pytest.mark.parametrize("engine", ["i8v", "bf16v"])
def test_filter_repeatable(vf, engine):
    """Race screen for the double-buffered LDS-DMA pipeline and the chunked
    launches: repeated searches over a corpus large enough to keep every CU busy
    give identical, correct lists."""
    xb = _rand(120000, 256, 47)
    xq = _rand(640, 256, 48)
    index = vf.IndexFlatIP(256)
    index.set_engine(engine)
    index.add(xb)
    D0, I0 = index.search(xq, 10)
    Dr, Ir = flat.knn_exact(xb, xq, 10, IP)
    assert not flat.mismatches(D0, I0, Dr, Ir, IP, xb, xq, strict=True)
    for _ in range(6):
        D, I = index.search(xq, 10)
        np.testing.assert_array_equal(I, I0)
        np.testing.assert_array_equal(D, D0)


@pytest.mark.parametrize("engine", ["i8v", "bf16v"])
def test_filter_selfjoin_offsets(vf, engine):
    """Self-join query tiles taken from the index's own filter plane at an
    offset, with and without self exclusion."""
    x = _rand(3000, 128, 49)
    index = vf.IndexFlatIP(128)
    index.set_engine(engine)
    index.add(x)
    Sr, Ir = flat.pgvector_cosine_topk(x, 12)
    S, I = index.selfjoin(12, q0=1000, nq=700)
    bad = flat.selfjoin_mismatches(S, I, Sr[1000:1700], Ir[1000:1700], x, np.arange(1000, 1700),
                                   strict=True)
    assert not bad, bad[:5]
    S2, I2 = index.selfjoin(12, q0=5, nq=300, exclude_self=False)
    assert (I2[:, 0] == np.arange(5, 305)).mean() > 0.99  # a row is its own best match


@pytest.mark.parametrize("metric,engine", FILTER_CASES)
def test_filter_matches_exact_engine(vf, metric, engine):
    """The filter-and-verify engine returns the exact lists: oracle parity (ids
    equal except documented ties) and the fp32 engine's ids on (nearly) every row
    — the two round their fp32 scores differently, so an exact near-tie may order
    differently."""
    xb = _rand(200000, 256, 60)
    xq = _rand(600, 256, 61)
    index = vf.IndexFlat(256, metric)
    index.add(xb)
    for k in (1, 4, 10, 12, 16, 28):
        index.set_engine("fp32")
        De, Ie = index.search(xq, k)
        index.set_engine(engine)
        D, I = index.search(xq, k)
        Dr, Ir = flat.knn_exact(xb, xq, k, metric)
        bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
        assert not bad, (k, bad[:5])
        assert (I == Ie).all(axis=1).mean() > 0.99
        np.testing.assert_allclose(D, De, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("engine", ["auto", "i8v", "bf16v"])
def test_filter_wide_k_inner_product(vf, engine):
    """Inner product past k = 28 (faiss's rule reads the 2k - 1 best: 64 and,
    past k = 32, 128 candidates per query — the select kernel, the 128-entry
    verification and emission): the filter engine answers (the statistics
    count the batch), exactly; raw lexicographic lists past 64 entries (a
    shard's half of a sharded k > 32 search) too."""
    from vsearch import _lib

    xb = _rand(200000, 256, 160)
    xq = _rand(600, 256, 161)
    index = vf.IndexFlatIP(256)
    index.set_engine(engine)
    index.add(xb)
    for k in (29, 32, 33, 50, 60, 64):
        _lib.filter_stats(reset=True)
        D, I = index.search(xq, k)
        nq, nfb = _lib.filter_stats(reset=True)
        assert nq == 600 and nfb <= 6, (k, nq, nfb)
        Dr, Ir = flat.knn_exact(xb, xq, k, IP)
        bad = flat.mismatches(D, I, Dr, Ir, IP, xb, xq, strict=True)
        assert not bad, (k, bad[:5])
    D, I = index.search(xq, 100, raw=True)
    Dr, Ir = flat.knn_lex(xb, xq, 100, IP)
    assert not flat.mismatches(D, I, Dr, Ir, IP, xb, xq, strict=True)


@pytest.mark.parametrize("metric,engine", FILTER_CASES)
def test_filter_falls_back_on_ties(vf, metric, engine):
    """Duplicated rows tie exactly, so the bound cannot separate the candidates:
    those queries are redone by the exact engine (on the device, gathered by a
    device-side list), and the results keep oracle parity."""
    from vsearch import _lib

    base = _rand(300, 64, 64)
    xb = np.concatenate([np.repeat(base[:20], 40, axis=0), base[20:]])  # 800 dup + 280
    xq = np.concatenate([base[:20] + 0.001 * _rand(20, 64, 65), _rand(300, 64, 66)])
    index = vf.IndexFlat(64, metric)
    index.set_engine(engine)
    index.add(xb)
    _lib.filter_stats(reset=True)
    D, I = index.search(xq, 10)
    nq, nfb = _lib.filter_stats(reset=True)
    assert nq == xq.shape[0] and nfb >= 20
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
    assert not bad, bad[:5]


def test_filter_every_query_falls_back(vf):
    """Every row tied 40 times and every query next to one: the whole batch goes
    to the exact redo (more flagged queries than one gathered tile, several query
    tiles) and keeps oracle parity."""
    from vsearch import _lib

    base = _rand(300, 64, 70)
    xb = np.repeat(base, 40, axis=0)
    xq = np.repeat(base, 4, axis=0)[:1024] + 0.001 * _rand(1024, 64, 71)
    index = vf.IndexFlatIP(64)
    index.add(xb)
    _lib.filter_stats(reset=True)
    D, I = index.search(xq, 10)
    nq, nfb = _lib.filter_stats(reset=True)
    assert nq == 1024 and nfb > 900
    Dr, Ir = flat.knn_exact(xb, xq, 10, IP)
    bad = flat.mismatches(D, I, Dr, Ir, IP, xb, xq, strict=True)
    assert not bad, bad[:5]


def test_filter_redo_runs_in_slot_windows(vf):
    """More flagged queries than one slot window of the exact redo (vs_api.hip
    run_gemm_rescored: lists capped at ~1 GB, here 11,136 slots at k = 20):
    every window is searched and rescored, queries of the second window included."""
    from vsearch import _lib

    base = _rand(300, 64, 74)
    xb = np.repeat(base, 40, axis=0)
    xq = np.tile(base, (41, 1))[:12288] + 0.001 * _rand(12288, 64, 75)
    index = vf.IndexFlatIP(64)
    index.add(xb)
    _lib.filter_stats(reset=True)
    D, I = index.search(xq, 20)
    nq, nfb = _lib.filter_stats(reset=True)
    assert nq == 12288 and nfb > 11200, nfb
    sample = np.r_[0:200, 11100:11400, 12088:12288]
    Dr, Ir = flat.knn_exact(xb, xq[sample], 20, IP)
    bad = flat.mismatches(D[sample], I[sample], Dr, Ir, IP, xb, xq[sample], strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("metric,engine", FILTER_CASES)
def test_filter_wide_check_settles_scattered_near_duplicates(vf, metric, engine):
    """40 near-copies of each base row, scattered over the corpus: the KF merged
    candidates are all copies, so the first check flags those queries; every lane
    list holds only one or two copies, so the wide check (all list entries below
    the list floors rescored) settles them without the exact engine; results keep
    oracle parity."""
    from vsearch import _lib

    base = _rand(60, 64, 80)
    xb = np.concatenate([np.repeat(base, 40, axis=0) + 1e-4 * _rand(2400, 64, 81),
                         _rand(4000, 64, 82)])
    xb = xb[np.random.default_rng(83).permutation(xb.shape[0])]
    xq = np.concatenate([base + 1e-4 * _rand(60, 64, 84), _rand(196, 64, 85)])
    index = vf.IndexFlat(64, metric)
    index.set_engine(engine)
    index.add(xb)
    _lib.filter_stats(reset=True)
    D, I = index.search(xq, 10)
    wide = _lib.filter_wide_stats()
    nq, n_exact = _lib.filter_stats(reset=True)
    assert nq == xq.shape[0]
    assert wide >= 60 and n_exact == 0, (metric, wide, n_exact)
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("metric", [IP, L2])
def test_filter_engines_agree(vf, metric):
    """Every filter engine of an fp32 index (the staged default, int8 alone,
    bf16 alone) returns the exact lists, for inner product and for L2 (whose
    int8 plane holds the augmented rows: L2 as an inner product)."""
    xb = _rand(20000, 192, 86)
    xq = _rand(300, 192, 87)
    index = vf.IndexFlat(192, metric)
    assert index.filter_planes == ("i8", "bf16")
    index.add(xb)
    Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
    for engine in ("auto", "bf16v", "i8v", "bf16v", "auto"):
        index.set_engine(engine)
        D, I = index.search(xq, 10)
        assert not flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True), engine


def test_l2_int8_plane_stays_out_of_other_metrics(vf):
    """The augmented int8 plane of an L2 index scores L2 only: the cosine
    self-join of the same index runs on its bf16 plane, exactly."""
    x = _rand(2000, 128, 90)
    index = vf.IndexFlatL2(128)
    index.add(x)
    S, I = index.selfjoin(12)
    Sr, Ir = flat.pgvector_cosine_topk(x, 12)
    bad = flat.selfjoin_mismatches(S, I, Sr, Ir, x, np.arange(2000), strict=True)
    assert not bad, bad[:5]


def _clustered(n, d, ncent, seed, cseed=5):
    """Unit-norm rows normalize(c[i % ncent] + 0.5 noise / sqrt(d)): clusters laid
    out periodically, like bench.py's clustered data."""
    c = np.random.default_rng(cseed).standard_normal((ncent, d))
    c /= np.linalg.norm(c, axis=1, keepdims=True)
    x = c[np.arange(n) % ncent] + 0.5 * np.random.default_rng(seed).standard_normal((n, d)) / d ** 0.5
    return (x / np.linalg.norm(x, axis=1, keepdims=True)).astype(np.float32)


def test_staged_engine_hands_clustered_queries_to_bf16(vf):
    """Clustered unit-norm rows: the int8 bound cannot separate a query's
    neighbours inside its cluster, so the staged engine hands (nearly) every
    query to the bf16 stage as a gathered batch, which settles them; results
    keep oracle parity, and the cosine self-join takes the same path."""
    from vsearch import _lib

    xb = _clustered(16384, 1536, 8, 91)
    xq = _clustered(300, 1536, 8, 92)
    index = vf.IndexFlatIP(1536)
    index.add(xb)
    _lib.filter_stats(reset=True)
    D, I = index.search(xq, 10)
    second = _lib.filter_second_stats()
    nq, n_exact = _lib.filter_stats(reset=True)
    assert nq == 300 and second > 200 and n_exact < 30, (second, n_exact)
    Dr, Ir = flat.knn_exact(xb, xq, 10, IP)
    bad = flat.mismatches(D, I, Dr, Ir, IP, xb, xq, strict=True)
    assert not bad, bad[:5]
    # the library has seen the int8 stage hand most queries on: the next search
    # starts on bf16 (nothing handed over), with the same exact results
    D2, I2 = index.search(xq, 10)
    second2 = _lib.filter_second_stats()
    _lib.filter_stats(reset=True)
    assert second2 == 0, second2
    assert not flat.mismatches(D2, I2, Dr, Ir, IP, xb, xq, strict=True)
    # the same rows through the cosine self-join (a 1000-student sub-range)
    S, J = index.selfjoin(15, q0=3000, nq=1000)
    Sr, Jr = flat.pgvector_cosine_topk(xb, 15, q_rows=np.arange(3000, 4000))
    bad = flat.selfjoin_mismatches(S, J, Sr, Jr, xb, np.arange(3000, 4000), strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("metric,k", [(IP, 10), (IP, 30), (flat.METRIC_L2, 10), (flat.METRIC_L2, 20)])
def test_select_heads_matches_list_merge(vf, metric, k, monkeypatch):
    """The first stage's candidate selection from the lane lists' heads
    (select_heads_kernel: the KF-th smallest head bounds the KF-th entry) gives
    the list merge's candidates: the same (D, I) and the same wide-check
    counts with VS_SELECT_HEADS=0, on rows with clusters of near-copies (lists
    whose every entry is below the bound) and exact against the oracle."""
    from vsearch import _lib

    rng = np.random.default_rng(77)
    d = 128
    xb = rng.uniform(-1, 1, (300_000, d)).astype(np.float32)
    hard = rng.uniform(-1, 1, (16, d)).astype(np.float32)
    pos = rng.choice(xb.shape[0], (16, 300), replace=False)
    for j in range(16):
        xb[pos[j]] = (hard[j] + 0.02 * rng.standard_normal((300, d))).astype(np.float32)
    xq = rng.uniform(-1, 1, (1024, d)).astype(np.float32)
    xq[:16] = hard + 0.01 * rng.standard_normal((16, d)).astype(np.float32)
    index = vf.IndexFlatL2(d) if metric == flat.METRIC_L2 else vf.IndexFlatIP(d)
    index.add(xb)
    out = {}
    for sel in ("1", "0"):
        monkeypatch.setenv("VS_SELECT_HEADS", sel)
        _lib.filter_stats(reset=True)
        D, I = index.search(xq, k)
        out[sel] = (D, I, _lib.filter_wide_stats())
        _lib.filter_stats(reset=True)
    assert np.array_equal(out["1"][1], out["0"][1])
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][2] == out["0"][2]
    rows = np.concatenate([np.arange(16), np.arange(16, 1024, 97)])
    Dr, Ir = flat.knn_exact(xb, xq[rows], k, metric)
    bad = flat.mismatches(out["1"][0][rows], out["1"][1][rows], Dr, Ir, metric, xb, xq[rows],
                          strict=True)
    assert not bad, bad[:5]


def test_deep_stage_few_queries_skinny(vf, monkeypatch):
    """A few hard queries in a large batch (40 of 4,096, each beside 200
    near-copies of its own direction): the int8 checks hand them on, and the
    deep bf16 stage for at most 64 queries runs skinny_plane_topk (one stream
    of the bf16 plane) instead of an x1 pass over a whole query tile.  Exact
    on every hard query and a sample of the rest, and the same results with
    the x1 deep pass (VS_SKINNY_DEEP=0)."""
    from vsearch import _lib

    rng = np.random.default_rng(123)
    d = 256
    xb = rng.uniform(-1, 1, (200_000, d)).astype(np.float32)
    hard = rng.uniform(-1, 1, (40, d)).astype(np.float32)
    pos = rng.choice(xb.shape[0], (40, 200), replace=False)
    for j in range(40):
        xb[pos[j]] = (hard[j] * (1.0 + 0.02 * rng.uniform(0, 1, (200, 1)))
                      + 0.01 * rng.standard_normal((200, d))).astype(np.float32)
    xq = rng.uniform(-1, 1, (4096, d)).astype(np.float32)
    hq = rng.choice(4096, 40, replace=False)
    xq[hq] = hard + 0.01 * rng.standard_normal((40, d)).astype(np.float32)
    index = vf.IndexFlatIP(d)
    index.add(xb)
    rows = np.unique(np.concatenate([hq, np.arange(0, 4096, 64)]))
    Dr, Ir = flat.knn_exact(xb, xq[rows], 10, IP)
    out = {}
    for skinny in ("1", "0"):
        monkeypatch.setenv("VS_SKINNY_DEEP", skinny)
        _lib.filter_stats(reset=True)
        D, I = index.search(xq, 10)
        second = _lib.filter_second_stats()
        _lib.filter_stats(reset=True)
        assert 1 <= second <= 64, second
        bad = flat.mismatches(D[rows], I[rows], Dr, Ir, IP, xb, xq[rows], strict=True)
        assert not bad, (skinny, bad[:5])
        out[skinny] = (D, I)
    assert np.array_equal(out["1"][1], out["0"][1])


@pytest.mark.parametrize("metric", [IP, flat.METRIC_L2])
def test_small_batches_through_the_filter_planes(vf, metric, monkeypatch):
    """Small batches (1 .. 64 queries) over an index of >= 2^18 rows run the
    staged engine with skinny passes (skinny_plane_topk over the int8 plane,
    then the bf16 plane and the fp32 rows for what it cannot settle): exact
    against the oracle, including queries beside 200 near-copies of their own
    direction that the int8 checks hand on, and the same labels as the exact
    streaming kernels (VS_SMALL_FILTER=0).  L2 calls of fewer than 20 queries
    keep faiss's sequential formula: their candidates are rescored as the
    rounded exact sum of (x - q)^2 (MODE_L2D)."""
    rng = np.random.default_rng(321)
    d = 128
    xb = rng.uniform(-1, 1, (300_000, d)).astype(np.float32)
    hard = rng.uniform(-1, 1, (6, d)).astype(np.float32)
    pos = rng.choice(xb.shape[0], (6, 200), replace=False)
    for j in range(6):
        xb[pos[j]] = (hard[j] * (1.0 + 0.02 * rng.uniform(0, 1, (200, 1)))
                      + 0.01 * rng.standard_normal((200, d))).astype(np.float32)
    index = vf.IndexFlatL2(d) if metric == flat.METRIC_L2 else vf.IndexFlatIP(d)
    index.add(xb)
    for nq in (1, 7, 32, 64):
        xq = rng.uniform(-1, 1, (nq, d)).astype(np.float32)
        nh = min(nq, 3)
        xq[:nh] = hard[:nh] + 0.01 * rng.standard_normal((nh, d)).astype(np.float32)
        monkeypatch.delenv("VS_SMALL_FILTER", raising=False)
        D, I = index.search(xq, 10)
        Dr, Ir = flat.knn_exact(xb, xq, 10, metric)
        # (L2 under 20 queries: faiss's sequential formula, rescored as the
        # rounded exact sum of (x - q)^2: strict as well)
        bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
        assert not bad, (nq, bad[:5])
        monkeypatch.setenv("VS_SMALL_FILTER", "0")
        D0, I0 = index.search(xq, 10)
        assert not flat.mismatches(D0, I0, Dr, Ir, metric, xb, xq), nq


def test_l2_small_calls_use_faiss_sequential_formula(vf):
    """faiss's IndexFlatL2 takes its sequential branch (dis = sum (x - y)^2) for
    calls of fewer than 20 queries and its BLAS branch (|x|^2 + |y|^2 - 2 x.y,
    clamped at 0) from 20 on.  A query equal to a stored row
    is at distance exactly 0 on the sequential branch; calls of 1, 5 and 19
    queries keep that (the filter engine rescores them as the rounded exact
    sum of (x - q)^2; with VS_SMALL_FILTER=0 the exact GEMV), and every
    distance is the direct sum's value within the fp32 contract; a call of 32
    queries is checked at the same tolerance (the BLAS formula's roundings)."""
    rng = np.random.default_rng(77)
    d = 128
    xb = rng.uniform(-1, 1, (300_000, d)).astype(np.float32)
    index = vf.IndexFlatL2(d)
    index.add(xb)
    import os
    for small in ("1", "0"):
        os.environ["VS_SMALL_FILTER"] = small
        try:
            for nq in (1, 5, 19, 32):
                src = rng.choice(xb.shape[0], nq, replace=False)
                xq = xb[src].copy()
                D, I = index.search(xq, 5)
                Dr, Ir = flat.knn_exact(xb, xq, 5, flat.METRIC_L2)
                assert not flat.mismatches(D, I, Dr, Ir, flat.METRIC_L2, xb, xq), (small, nq)
                assert (I[:, 0] == src).all(), (small, nq)
                if nq < 20:
                    assert (D[:, 0] == 0.0).all(), (small, nq, D[:, 0])
        finally:
            del os.environ["VS_SMALL_FILTER"]
