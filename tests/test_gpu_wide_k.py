"""GPU parity of searches past one 64-entry page: any k, as faiss-cpu's
IndexFlat::search answers it (the live tool's k is the agent's,
/root/reference/src/recommendation_api/mcp_book_server.py:115,142; LangChain
passes fetch_k straight to index.search under a filter).  These searches run
the paged exact engine (vs_api.hip run_paged): the exact fp32 / bf16 kernels
page through each query's lexicographic (key, row) order 64 entries at a time.

Acceptance: the fp32 contract of the north star (labels equal except ties
within, and scores within, 1e-5 * max(1, |s|); oracle/flat.py mismatches_vec
for the large results), labels and scores bit for bit against the C faiss-heap
restatement on integer rows (exact scores), and the strict proven-candidate
check at 1M x 1536."""

import ctypes

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


def _rand(n, d, seed, kind="normal"):
    rng = np.random.default_rng(seed)
    if kind == "normal":
        return rng.standard_normal((n, d)).astype(np.float32)
    return rng.integers(-2, 3, size=(n, d)).astype(np.float32)


def _check(D, I, xb, xq, k, metric, raw=False):
    if raw:
        Dr, Ir = flat.knn_lex(xb, xq, k, metric)
    else:
        Dr, Ir = flat.knn_exact(xb, xq, k, metric)
    bad = flat.mismatches_vec(D, I, Dr, Ir, metric, xb, xq)
    assert not bad, bad[:5]


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("k", [65, 100, 500, 2048])
def test_any_k_against_oracle(vf, k, metric, dtype):
    """k in {65, 100, 500, 2048}, B in {1, 37, 4096}: B = 1 on the GEMV (fp32
    inner product; fp32 L2 calls under 20 queries take faiss's sequential
    formula), the MFMA GEMM otherwise; bf16 storage against the oracle over the
    bf16-rounded rows and queries."""
    d = 32
    xb = _rand(6000, d, 100 + k)
    index = vf.IndexFlat(d, metric, dtype=dtype)
    index.add(xb)
    xr = flat.round_bf16(xb) if dtype == "bf16" else xb
    for nq in (1, 37, 4096):
        xq = _rand(nq, d, 200 + nq)
        D, I = index.search(xq, k)
        assert D.shape == (nq, k)
        rq = flat.round_bf16(xq) if dtype == "bf16" else xq
        _check(D, I, xr, rq, k, metric)


@pytest.mark.parametrize("metric", [L2, IP])
def test_any_k_padding_past_ntotal(vf, metric):
    """k > ntotal: (neutral, -1) past the rows there are (faiss's heap padding),
    on every kernel (B = 1, 5 and 40)."""
    for n, k in ((70, 100), (1000, 2048)):
        xb = _rand(n, 16, 300 + n)
        index = vf.IndexFlat(16, metric)
        index.add(xb)
        for nq in (1, 5, 40):
            xq = _rand(nq, 16, 301 + nq)
            D, I = index.search(xq, k)
            assert (I[:, n:] == -1).all() and (D[:, n:] == flat.neutral(metric)).all()
            assert (np.sort(I[:, :n], axis=1) == np.arange(n)).all()
            _check(D, I, xb, xq, k, metric)


@pytest.mark.parametrize("metric", [L2, IP])
@pytest.mark.parametrize("k", [65, 100, 300, 599, 700])
def test_any_k_ties_match_faiss_heap(vf, metric, k):
    """Tie-heavy integer rows (d = 3: long runs of equal scores): labels and
    scores equal the C restatement of faiss's heaps exactly.  Inner product's
    rule reads the k-th key's run of ties up to 2k - 1 entries, so the pages
    continue past k while the run fills them."""
    xb = _rand(600, 3, 12, "int")
    for nq in (1, 7, 40):
        xq = _rand(nq, 3, 13 + nq, "int")
        index = vf.IndexFlat(3, metric)
        index.add(xb)
        D, I = index.search(xq, k)
        Dc, Ic = cfaiss.knn_seq(xb, xq, k, metric)
        np.testing.assert_array_equal(I, Ic)
        np.testing.assert_array_equal(D, Dc)


@pytest.mark.parametrize("nq", [1, 5, 300])
@pytest.mark.parametrize("k", [100, 300])
@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_any_k_duplicate_rows(vf, nq, k, dtype):
    """500 copies of one row (a re-ingested book, book_vector/main.py:148)
    around the queries: the copies' run of equal keys spans several pages and
    faiss's rule keeps the right k of their labels (descending)."""
    d = 64
    xb = _rand(6000, d, 71)
    dup = _rand(1, d, 72)[0]
    pos = np.random.default_rng(73).choice(6000, 500, replace=False)
    xb[pos] = dup
    xq = _rand(nq, d, 74) * 0.05 + dup
    index = vf.IndexFlat(d, IP, dtype=dtype)
    index.add(xb)
    D, I = index.search(xq, k)
    if dtype == "bf16":
        xb, xq = flat.round_bf16(xb), flat.round_bf16(xq)
    Dc, Ic = cfaiss.knn_seq(xb, xq, k, IP)
    np.testing.assert_array_equal(I, Ic)
    np.testing.assert_allclose(D, Dc, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
@pytest.mark.parametrize("k", [65, 200])
def test_any_k_raw_lexicographic(vf, k, dtype):
    """VS_RAW_ORDER past 64 entries (a shard's half of a sharded k > 32 search:
    2k - 1 raw entries): integer rows, the lexicographic order bit for bit."""
    xb = _rand(900, 4, 81, "int")
    for nq in (1, 7, 200):
        xq = _rand(nq, 4, 82, "int")
        index = vf.IndexFlat(4, IP, dtype=dtype)
        index.add(xb)
        D, I = index.search(xq, k, raw=True)
        Dr, Ir = flat.knn_lex(xb, xq, k, IP)
        np.testing.assert_array_equal(I, Ir)
        np.testing.assert_array_equal(D, Dr)


@pytest.mark.parametrize("metric", [L2, IP])
def test_any_k_bf16_tombstones(vf, metric, monkeypatch):
    """A bf16 index with tombstoned removals (C5's interleaved remove/add):
    the pages skip the NaN rows and their labels come out as faiss positions
    among the live rows, for k = 150 and a raw k = 200."""
    monkeypatch.setenv("VS_PACK_DEN", "16")
    d = 96
    xb = _rand(8000, d, 11)
    index = vf.IndexFlat(d, metric, dtype="bf16")
    index.add(xb)
    xr = flat.round_bf16(xb)
    rng = np.random.default_rng(12)
    for r in range(2):
        rm = rng.choice(xr.shape[0], 60, replace=False)
        assert index.remove_ids(rm) == 60
        xr, _ = flat.remove_ids(xr, rm)
        add = _rand(50, d, 20 + r)
        index.add(add)
        xr = np.concatenate([xr, flat.round_bf16(add)])
        for nq in (1, 40):
            xq = _rand(nq, d, 30 + r + nq)
            rq = flat.round_bf16(xq)
            D, I = index.search(xq, 150)
            _check(D, I, xr, rq, 150, metric)
            D, I = index.search(xq, 200, raw=True)
            _check(D, I, xr, rq, 200, metric, raw=True)


@pytest.mark.parametrize("dtype", ["f32", "bf16"])
def test_any_k_selfjoin(vf, dtype):
    """The student self-join (pgvector's ORDER BY <=> LIMIT k has no k limit):
    k = 100 and 300, self excluded, and a similarity threshold."""
    x = _rand(700, 48, 8)
    index = vf.IndexFlatIP(48, dtype=dtype)
    index.add(x)
    xr = flat.round_bf16(x) if dtype == "bf16" else x
    for k in (100, 300):
        S, I = index.selfjoin(k)
        Sr, Ir = flat.pgvector_cosine_topk(xr, k)
        bad = flat.selfjoin_mismatches(S, I, Sr, Ir, xr, np.arange(700))
        assert not bad, bad[:5]
    S, I = index.selfjoin(120, q0=50, nq=80, min_sim=0.05)
    Sr, Ir = flat.pgvector_cosine_topk(xr, 120, q_rows=np.arange(50, 130), min_sim=0.05)
    bad = flat.selfjoin_mismatches(S, I, Sr, Ir, xr, np.arange(50, 130))
    assert not bad, bad[:5]


@pytest.mark.parametrize("metric", [L2, IP])
def test_merge_topk_any_k(vf, metric):
    """vs_merge_topk past 64 entries: three shards' raw lists (2k - 1 for inner
    product) merged on the GPU equal one index over all rows, k = 100 and 300."""
    torch = pytest.importorskip("torch")
    from vsearch import _lib

    xb = _rand(4000, 32, 21)
    xq = _rand(50, 32, 22)
    for k in (100, 300):
        kin = 2 * k - 1 if metric == IP else k
        parts = []
        for lo, hi in ((0, 1000), (1000, 2500), (2500, 4000)):
            idx = vf.IndexFlat(32, metric)
            idx.add(xb[lo:hi])
            idx.set_id_base(lo)
            parts.append(idx.search(xq, kin, raw=True))
        Dp = torch.from_numpy(np.stack([p[0] for p in parts])).cuda()
        Ip = torch.from_numpy(np.stack([p[1] for p in parts])).cuda()
        D = torch.empty((50, k), dtype=torch.float32, device="cuda")
        I = torch.empty((50, k), dtype=torch.int64, device="cuda")
        _lib.check(_lib.load().vs_merge_topk(
            ctypes.c_void_p(Dp.data_ptr()), ctypes.c_void_p(Ip.data_ptr()), 3, 50, kin, k, metric,
            ctypes.c_void_p(D.data_ptr()), ctypes.c_void_p(I.data_ptr()), None))
        torch.cuda.synchronize()
        _check(D.cpu().numpy(), I.cpu().numpy(), xb, xq, k, metric)


def test_store_similarity_search_k100(golden, golden_vectors):
    """FAISS.similarity_search(query, k=100) through the drop-in store (the
    reference's catalogue, L2 default): the documents in the oracle's order;
    and a filtered search, whose fetch_k = 150 goes straight to index.search."""
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, _ = golden
    xb, _, _ = golden_vectors
    emb = SynthEmbeddings()
    store = vlc.FAISS.from_texts(inputs["book_texts"], emb, metadatas=inputs["book_metadata"])
    pos = {m["book_id"]: i for i, m in enumerate(inputs["book_metadata"])}
    for kw in inputs["keywords"][:8]:
        docs = store.similarity_search_with_score(kw, k=100)
        assert len(docs) == 100
        I = np.array([[pos[d.metadata["book_id"]] for d, _ in docs]], dtype=np.int64)
        D = np.array([[s for _, s in docs]], dtype=np.float32)
        xq = np.asarray(emb.embed_query(kw), dtype=np.float32)[None, :]
        _check(D, I, xb, xq, 100, L2)
    genre = inputs["book_metadata"][0]["genre"]
    docs = store.similarity_search(inputs["keywords"][0], k=10, filter={"genre": genre},
                                   fetch_k=150)
    assert docs and all(d.metadata["genre"] == genre for d in docs)


@pytest.mark.parametrize("metric", [L2, IP])
def test_any_k_large_sampled(vf, metric):
    """1M x 1536 (C2's corpus), B = 4096, k = 100: sampled queries from the
    first and last query tiles against proven candidate sets (the 256 best by
    fp32 sgemm, margin-checked, rescored in fp64) with the fp32 contract."""
    from vsearch.synth import synthetic_rows

    n, d, k = 1_000_000, 1536, 100
    index = vf.IndexFlat(d, metric)
    index.reserve(n)
    index.add_synthetic(n, seed=1234)
    xq = synthetic_rows(50_000_000, 4096, d, 5678)
    D, I = index.search(xq, k)
    assert (I >= 0).all() and (I < n).all()
    if metric == L2:
        assert (np.diff(D, axis=1) >= 0).all()
    else:
        assert (np.diff(D, axis=1) <= 0).all()
    sample = [0, 1, 127, 4095]
    from helpers import proven_candidates

    K = 2 * k - 1 if metric == IP else k
    cands = proven_candidates(index, xq[sample], metric, n, K, m=256)
    for row, q in enumerate(sample):
        assert_against_candidates(D[q], I[q], cands[row], metric, k, d, strict=False)


@pytest.mark.parametrize("metric", [L2, IP])
def test_staged_engine_past_64(vf, metric):
    """k past one page through the staged filter-and-verify engine (up to 1024
    candidates per query: inner product k <= 512, L2 k <= 1023): small batches
    over >= 2^18 rows (the int8 plane's skinny pass) and a large batch (the x1
    pass), STRICT parity on every query (the answers are exact roundings of
    rescored scores); k = 1100 goes past the staged engine to the paged one."""
    from vsearch import _lib

    n, d = 300_000, 64
    xb = _rand(n, d, 900)
    index = vf.IndexFlat(d, metric)
    index.add(xb)
    ks = (100, 200, 700) if metric == L2 else (65, 100, 300)
    for nq in (1, 8, 300):
        xq = _rand(nq, d, 901 + nq)
        for k in ks:
            _lib.filter_stats(reset=True)
            D, I = index.search(xq, k)
            fq, _ = _lib.filter_stats(reset=True)
            assert fq == nq, (nq, k, fq)  # the staged engine answered
            Dr, Ir = flat.knn_exact(xb, xq, k, metric)
            bad = flat.mismatches(D, I, Dr, Ir, metric, xb, xq, strict=True)
            assert not bad, (nq, k, bad[:3])
    xq = _rand(40, d, 999)
    D, I = index.search(xq, 1100)
    _check(D, I, xb, xq, 1100, metric)
