"""GPU: the filter pass's dump launches (vs_gemm_x1.hip header).

A pass of an int8 or bf16 inner-product filter over splits of at least 16
tiles runs its first launch as a list launch, sets each query's cut from those
lists (x1_qcut), and runs the rest as dump launches whose blocks below the cut
x1_replay folds into the lists.  The small parity tests never reach that
length (their splits are a few tiles), so these searches are sized for it:
4,096 queries (16 query tiles, 32 splits) over 300,000 rows (37 tiles per
split, launches of 8 tiles: one list launch + four dump launches in three
segments), checked STRICTLY against the
fp64 oracle on 512 sampled queries (every query tile), with the dump counters
showing that dump launches ran.  Also: lane lists that run out of dump slots
(150,000 ever-better copies of a row next to the queries: ~230 candidate rows
per list and segment > 128 slots) hand their queries to the next stage and the answer stays exact;
the bf16 plane's dump form; and the cosine self-join (C4's path), which keeps
list launches."""

import numpy as np
import pytest

from oracle import flat

pytestmark = pytest.mark.gpu

IP = flat.METRIC_INNER_PRODUCT
N, D_, B = 300_000, 128, 4096
SAMPLE = np.array(sorted({q for t in range(16) for q in range(256 * t, 256 * t + 256, 8)}))


@pytest.fixture(scope="module")
def lib():
    """Launches of 8 tiles per workgroup (VS_X1_CHUNK_TILES, read at every
    search): 37-tile splits become a 5-launch pass, which has dump launches
    (a pass needs at least 4; at the default 64 tiles that takes ~1.6M rows)."""
    import os

    from vsearch import _lib

    assert _lib.device_count() >= 1
    old = os.environ.get("VS_X1_CHUNK_TILES")
    os.environ["VS_X1_CHUNK_TILES"] = "8"
    yield _lib
    if old is None:
        del os.environ["VS_X1_CHUNK_TILES"]
    else:
        os.environ["VS_X1_CHUNK_TILES"] = old


def _search_checked(lib, xb, xq, k, engine="auto", metric=IP):
    from vsearch import faiss as vfaiss

    index = vfaiss.IndexFlat(xb.shape[1], metric)
    index.add(xb)
    index.set_engine(engine)
    lib.filter_stats(reset=True)
    D, I = index.search(xq, k)
    dumps, over = lib.filter_dump_stats()
    fq, ff = lib.filter_stats(reset=True)
    Dr, Ir = flat.knn_exact(xb, xq[SAMPLE], k, metric)
    bad = flat.mismatches(D[SAMPLE], I[SAMPLE], Dr, Ir, metric, xb, xq[SAMPLE], strict=True)
    assert not bad, bad[:5]
    return dumps, over, fq, ff


@pytest.mark.parametrize("kind", ["uniform", "normal"])
def test_dump_launches_l2_augmented(lib, kind):
    """L2 through the int8 plane's augmented rows (L2 as an inner product): the
    same list / dump launches, cuts and replays as an inner-product pass, the
    lane lists mapped to L2 keys after it; exact on the sample, dump launches
    ran, no list out of slots and no query left to the exact engine."""
    rng = np.random.default_rng(41)
    if kind == "uniform":
        xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
        xq = rng.uniform(-1, 1, (B, D_)).astype(np.float32)
    else:
        xb = rng.standard_normal((N, D_)).astype(np.float32)
        xq = rng.standard_normal((B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, 10, engine="i8v", metric=flat.METRIC_L2)
    assert fq == B and dumps > 0, (dumps, over)
    if kind == "uniform":  # rows of one scale: the launch's factor bound is tight
        assert over == 0 and ff == 0, (dumps, over, ff)
    # Gaussian rows at d = 128: max|x| (the int8 scale) varies ~2x between rows, so
    # the launch's largest factor passes many more rows than reach a list and
    # some lists run out of slots; their queries go to the next stage (exactly)


@pytest.mark.parametrize("k", [1, 10, 28])
def test_dump_launches_uniform_rows(lib, k):
    rng = np.random.default_rng(31 + k)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    xq = rng.uniform(-1, 1, (B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, k)
    assert fq == B
    assert dumps > 0 and over == 0, (dumps, over)


def test_dump_launches_clustered_unit_rows(lib):
    """Embedding-like rows (unit norm, 64 centroids): the int8 cut sits close
    to the top, the bf16 stage takes what int8 cannot settle."""
    rng = np.random.default_rng(5)
    c = rng.standard_normal((64, D_)).astype(np.float32)
    xb = c[rng.integers(0, 64, N)] + 0.5 * rng.standard_normal((N, D_)).astype(np.float32)
    xb /= np.linalg.norm(xb, axis=1, keepdims=True)
    xq = c[rng.integers(0, 64, B)] + 0.5 * rng.standard_normal((B, D_)).astype(np.float32)
    xq /= np.linalg.norm(xq, axis=1, keepdims=True)
    dumps, over, fq, _ = _search_checked(lib, xb, xq, 10)
    assert fq == B and dumps > 0


def test_dump_slot_overflow_hands_queries_on(lib):
    """150,000 scaled copies of one row beside every query, each better than
    every copy at a lower row: in a dump launch a lane list meets ~256 of them
    below its cut and its own last entry — more candidate rows than its 128 dump
    slots.  The query is failed by the verification (cut = -FLT_MAX), the bf16
    stage's bound cannot separate thousands of copies either, and the exact
    stage answers.  The copies' scores are spaced ~2e-6 apart (relative): far
    above the exact stage's fp32 rounding, whose candidate set decides which
    rows get rescored (copies spaced below it — a factor of 1 + 1e-3 pos / N,
    round 5's first form — tie inside that rounding, and its top-KF candidates
    need not hold the fp64 top-k: the north star's 1e-5 tolerance, not the
    strict window)."""
    rng = np.random.default_rng(77)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    dup = rng.uniform(-1, 1, D_).astype(np.float32)
    pos = np.sort(rng.choice(N, 150_000, replace=False))
    xb[pos] = dup[None, :] * (1.0 + 0.3 * pos[:, None] / N).astype(np.float32)
    xq = (dup[None, :] + 0.3 * rng.uniform(-1, 1, (B, D_))).astype(np.float32)
    dumps, over, fq, _ = _search_checked(lib, xb, xq, 10)
    assert over > 0, (dumps, over)


@pytest.mark.parametrize("engine", ["auto", "i8v"])
def test_dense_near_ties_reach_the_exact_stream(lib, engine):
    """Round 5's first form of the test above: the copies' factors 1 + 1e-3 pos / N
    put them ~7e-9 apart (relative), far inside the fp32 GEMM's rounding, so no
    fp32 candidate list of the last stage holds a provable top-k (thousands of
    copies inside its bound).  The last stage proves its candidates with the
    fp32 GEMM's own bound and hands what it cannot prove to the exact-key stream
    (vs_exact.hip: every row ranked by the rescoring's key): STRICT parity."""
    from vsearch import faiss as vfaiss

    rng = np.random.default_rng(77)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    dup = rng.uniform(-1, 1, D_).astype(np.float32)
    pos = np.sort(rng.choice(N, 150_000, replace=False))
    xb[pos] = dup[None, :] * (1.0 + 1e-3 * pos[:, None] / N).astype(np.float32)
    xq = (dup[None, :] + 0.3 * rng.uniform(-1, 1, (B, D_))).astype(np.float32)
    index = vfaiss.IndexFlat(D_, IP)
    index.add(xb)
    index.set_engine(engine)
    lib.filter_stats(reset=True)
    D, I = index.search(xq, 10)
    streamed = lib.filter_exact_stats()
    lib.filter_stats(reset=True)
    assert streamed > 0
    Dr, Ir = flat.knn_exact(xb, xq[SAMPLE], 10, IP)
    bad = flat.mismatches(D[SAMPLE], I[SAMPLE], Dr, Ir, IP, xb, xq[SAMPLE], strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("k", [40, 100])
def test_dense_near_ties_past_32_exact_pages(lib, k):
    """The same near-ties at inner product k = 40 / 100 (79 / 199 candidates,
    past the 64 that one exact page holds): what no filter stage settles runs
    the paged engine over exact-key pages (vs_exact.hip with a floor per query:
    every key the rescoring's own) instead of the fp32 GEMM's
    pages, so the answer is STRICT here too."""
    from vsearch import faiss as vfaiss

    rng = np.random.default_rng(78)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    dup = rng.uniform(-1, 1, D_).astype(np.float32)
    pos = np.sort(rng.choice(N, 150_000, replace=False))
    xb[pos] = dup[None, :] * (1.0 + 1e-3 * pos[:, None] / N).astype(np.float32)
    xq = (dup[None, :] + 0.3 * rng.uniform(-1, 1, (B, D_))).astype(np.float32)
    index = vfaiss.IndexFlat(D_, IP)
    index.add(xb)
    lib.filter_stats(reset=True)
    D, I = index.search(xq, k)
    streamed = lib.filter_exact_stats()
    lib.filter_stats(reset=True)
    assert streamed > 0
    Dr, Ir = flat.knn_exact(xb, xq[SAMPLE], k, IP)
    bad = flat.mismatches(D[SAMPLE], I[SAMPLE], Dr, Ir, IP, xb, xq[SAMPLE], strict=True)
    assert not bad, bad[:5]


def test_dump_launches_queries_pointing_away(lib):
    """Every inner product below 0 (rows in [0, 1), queries in [-1, 0)): the
    lists' floors are above 0, where the largest row factor bounds nothing (a
    row with a negative sum scores highest with its SMALLEST factor).  The dump
    launches take their threshold from the launch's smallest factor there, so
    the lists stay within their slots and the int8 stage settles the queries
    instead of handing the whole batch on; the answer is exact either way."""
    rng = np.random.default_rng(23)
    xb = rng.uniform(0, 1, (N, D_)).astype(np.float32)
    xq = -rng.uniform(0, 1, (B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, 10, engine="i8v")
    assert fq == B and dumps > 0
    assert over <= B * 128 * 0.01, (dumps, over)  # < 1 % of the 128 lane lists per query
    assert ff <= B // 20, ff


def test_dump_launches_bf16_plane(lib):
    rng = np.random.default_rng(9)
    xb = rng.standard_normal((N, D_)).astype(np.float32)
    xq = rng.standard_normal((B, D_)).astype(np.float32)
    dumps, over, fq, _ = _search_checked(lib, xb, xq, 10, engine="bf16v")
    assert dumps > 0 and over == 0


def test_cosine_selfjoin_keeps_list_launches(lib):
    """C4's path at reduced size: 300,000 students (65,536-student chunks, 32
    splits of 37 tiles), cosine top-15 excluding self, strict on 256 rows.
    The cosine pass has no dump form (its relative bound puts the cut behind
    the lists' own floors: this d = 128 self-join made 31 dumps per list when
    it had one), so it runs list launches only."""
    from vsearch import faiss as vfaiss

    rng = np.random.default_rng(13)
    x = rng.standard_normal((N, D_)).astype(np.float32)
    index = vfaiss.IndexFlatIP(D_)
    index.add(x)
    lib.filter_stats(reset=True)
    S, I = index.selfjoin(15)
    dumps, over = lib.filter_dump_stats()
    lib.filter_stats(reset=True)
    assert dumps == 0 and over == 0
    rows = np.array(sorted({r for c in range(0, N, 65536) for r in (c, c + 1, c + 65535)
                            if r < N} | set(range(0, N, N // 200))))
    Sr, Ir = flat.pgvector_cosine_topk(x, 15, q_rows=rows)
    bad = flat.selfjoin_mismatches(S[rows], I[rows], Sr, Ir, x, rows, strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("metric", [IP, flat.METRIC_L2])
def test_hybrid_single_launch(lib, metric, monkeypatch):
    """A pass of one launch (C2's shape: 37 tiles per workgroup here) runs as a
    hybrid launch (vs_gemm_x1.hip, HYB): its first quarter of tiles keeps lists
    in registers, the rest dumps below each list's own last entry, and the
    replay after it admits the dumps: exact on the sample, dumps made, no list
    out of its slots, nothing left to a later stage."""
    monkeypatch.setenv("VS_X1_CHUNK_TILES", "64")
    monkeypatch.setenv("VS_X1_HYB", "1")  # off by default (vs_gemm_x1.hip, x1_hybrid_on)
    monkeypatch.setenv("VS_X1_SPLIT", "0")  # a split pass would take the pass instead
    rng = np.random.default_rng(57)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    xq = rng.uniform(-1, 1, (B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, 10, engine="i8v", metric=metric)
    assert fq == B and dumps > 0 and over == 0 and ff == 0, (dumps, over, ff)


@pytest.mark.parametrize("metric", [IP, flat.METRIC_L2])
def test_split_pass(lib, metric, monkeypatch):
    """A pass of one launch (C2's shape: 37 tiles per workgroup here) as a split
    pass (VS_X1_SPLIT=4, vs_gemm_x1.hip x1_launch): a list launch over the first
    quarter of every workgroup's tiles, the cuts, one dump launch over the rest
    and one replay: exact on the sample, dumps made, no list out of its slots,
    nothing left to a later stage."""
    monkeypatch.setenv("VS_X1_CHUNK_TILES", "64")
    monkeypatch.setenv("VS_X1_SPLIT", "4")
    rng = np.random.default_rng(58)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    xq = rng.uniform(-1, 1, (B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, 10, engine="i8v", metric=metric)
    assert fq == B and dumps > 0 and over == 0 and ff == 0, (dumps, over, ff)


def test_cosine_selfjoin_dump_form(lib, monkeypatch):
    """The int8 cosine's dump form (VS_X1_COSDUMP=1: the folded factors s_x / |x|
    in the launch-wide threshold, the same keys as its list launches) on the
    C4-shaped self-join above: exact on the sampled students, dump launches ran."""
    from vsearch import faiss as vfaiss

    monkeypatch.setenv("VS_X1_COSDUMP", "1")
    rng = np.random.default_rng(14)
    x = rng.standard_normal((N, D_)).astype(np.float32)
    index = vfaiss.IndexFlatIP(D_)
    index.add(x)
    lib.filter_stats(reset=True)
    S, I = index.selfjoin(15)
    dumps, over = lib.filter_dump_stats()
    lib.filter_stats(reset=True)
    assert dumps > 0
    rows = np.array(sorted({r for c in range(0, N, 65536) for r in (c, c + 1, c + 65535)
                            if r < N} | set(range(0, N, N // 200))))
    Sr, Ir = flat.pgvector_cosine_topk(x, 15, q_rows=rows)
    bad = flat.selfjoin_mismatches(S[rows], I[rows], Sr, Ir, x, rows, strict=True)
    assert not bad, bad[:5]


@pytest.mark.parametrize("den,seg", [(8, "0"), (16, "1"), (32, "1")])
def test_split_pass_segments(lib, monkeypatch, den, seg):
    """Split passes (one launch per workgroup's tiles: 300,000 rows, 37 tiles
    per split at the default 64-tile launches): a list launch over 1/den of
    the tiles, then one dump launch, or (VS_X1_SPLITSEG=1) dump launches over
    doubling part ranges with a replay after each.  Strict on the sample, no
    list out of slots, nothing handed to the next stage."""
    monkeypatch.setenv("VS_X1_CHUNK_TILES", "64")
    monkeypatch.setenv("VS_X1_SPLIT", str(den))
    monkeypatch.setenv("VS_X1_SPLITSEG", seg)
    rng = np.random.default_rng(17)
    xb = rng.uniform(-1, 1, (N, D_)).astype(np.float32)
    xq = rng.uniform(-1, 1, (B, D_)).astype(np.float32)
    dumps, over, fq, ff = _search_checked(lib, xb, xq, 10, engine="i8v")
    assert fq == B and dumps > 0 and over == 0 and ff == 0, (dumps, over, ff)
