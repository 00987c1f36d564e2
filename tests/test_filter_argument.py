"""CPU model of the filter-and-verify exactness argument (DESIGN.md §4.2 and the
wide check, vs_gemm_x3.hip verify_rescore_kernel / verify_wide_kernel).

The kernels keep, per query, P lane lists of the L lexicographically smallest
(approximate key, row) pairs of the rows each list sees.  Both checks rescore a
candidate set S exactly and accept when  T - B > E_M,  where every row outside S
has approximate key >= T, |approx - exact| <= B for every row, and E_M is the
M-th smallest exact key in S.  This model draws exact keys with near-duplicate
clusters, perturbs them by at most B, builds the lane lists, applies both
checks, and asserts that every accepted query's top-M (ties broken by row) is the
exact one.  It is a statement about the algorithm, not about the GPU code: the
GPU tests check the kernels against the oracle."""

import numpy as np


def _lane_lists(a, P, L, rng):
    """Rows dealt to P lists (random ownership, as tiles interleave rows); each
    list keeps its L lexicographically smallest (approx key, row)."""
    owner = rng.integers(0, P, size=a.shape[0])
    lists = []
    for p in range(P):
        rows = np.nonzero(owner == p)[0]
        order = np.lexsort((rows, a[rows]))[:L]
        lists.append(rows[order])
    return lists


def _accept(S, T, e, B, M):
    if len(S) < M:
        return False, None
    S = np.asarray(sorted(S))
    order = np.lexsort((S, e[S]))
    top = S[order]
    return bool(T - B > e[top[M - 1]]), top[:M]


def _check_query(e, a, B, P, L, KF, M, rng):
    lists = _lane_lists(a, P, L, rng)
    full = [lst for lst in lists if len(lst) == L]
    floor = min((a[lst[-1]] for lst in full), default=np.inf)
    entries = np.concatenate(lists)
    # first check: the KF merged candidates; T = min(KF-th key, list floors)
    merged = entries[np.lexsort((entries, a[entries]))][:KF]
    T1 = min(a[merged[-1]] if len(merged) == KF else np.inf, floor)
    ok1, top1 = _accept(list(merged), T1, e, B, M)
    # wide check: every list entry below the list floors
    wide = [r for r in entries if a[r] < floor] if np.isfinite(floor) else list(entries)
    ok2, top2 = _accept(wide, floor, e, B, M)
    exact = np.lexsort((np.arange(e.shape[0]), e))[:M]
    for ok, top in ((ok1, top1), (ok2, top2)):
        if ok:
            np.testing.assert_array_equal(top, exact)
    return ok1, ok2


def test_filter_and_wide_checks_are_exact_when_they_accept():
    rng = np.random.default_rng(2024)
    B = 1e-3
    first = wide = 0
    n_q = 60
    for q in range(n_q):
        n = 3000
        e = rng.standard_normal(n).astype(np.float64)
        # a cluster of near-duplicates at the top (keys: smaller is better) for
        # most queries, as clustered embeddings have: 40 rows within 4 B
        if q % 4:
            e[rng.choice(n, 40, replace=False)] = -5.0 + rng.uniform(0, 4 * B, 40)
        a = e + rng.uniform(-B, B, n)  # |approx - exact| <= B
        ok1, ok2 = _check_query(e, a, B, P=32, L=16, KF=32, M=19, rng=rng)
        first += ok1
        wide += ok2
    # the wide check settles what the KF-candidate check cannot
    assert wide > first
    assert wide == n_q


def test_wide_check_rejects_a_list_full_of_ties():
    """Exact duplicates that fill one lane list pull its floor onto their key: the
    wide check must refuse (the exact engine then redoes the query)."""
    rng = np.random.default_rng(7)
    B = 1e-3
    n = 500
    e = rng.standard_normal(n)
    e[:40] = 5.0  # 40 exact ties, all owned by one list below
    a = e.copy()
    lists = [np.arange(16)] + [np.arange(40 + 16 * p, 56 + 16 * p) for p in range(20)]
    floor = min(a[lst[-1]] for lst in lists)
    entries = np.concatenate(lists)
    wide = [r for r in entries if a[r] < floor]
    ok, _ = _accept(wide, floor, e, B, 19)
    assert not ok


# ---------------------------------------------------------------------------
# The int8 filter plane's bound (vs_gemm_x1.hip quantize_i8_kernel,
# bound_key, make_bound_args): codes c = rint(x / s) clamped to +-127 with one
# fp32 scale s = max|x| / 127 per row; the kernel's approximate inner product is
# fl(fl(float(c_q . c_x)) * fl(s_q * s_x)) (exact int32 sum).  This restates
# the arithmetic in numpy (fp32 where the kernel is fp32) and checks
# |approx - x.q| <= B for every (query, row) pair, including rows with outliers,
# tiny and zero rows, and the cosine form with folded inverse norms.

_U = 2.0 ** -24
_GAM_I8 = 6.0 * _U


def _quantize_i8(x):
    x = np.asarray(x, np.float32)
    m = np.abs(x).max(axis=1)
    s = (m / np.float32(127.0)).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        c = np.where(s[:, None] > 0, np.rint(x / s[:, None]), 0.0)
    c = np.clip(c, -127, 127).astype(np.int64)
    r = x.astype(np.float64) - s[:, None].astype(np.float64) * c
    rn2 = np.nextafter((r * r).sum(axis=1).astype(np.float32), np.float32(np.inf))
    return c, s, rn2


def _rows(rng, n, d):
    x = rng.uniform(-1, 1, (n, d)).astype(np.float32)
    x[1] = 0.0                                     # zero row
    x[2] *= 1e-30                                  # tiny row
    x[3, 5] = 40.0                                 # one outlier element
    x[4] = rng.standard_normal(d).astype(np.float32) / np.sqrt(d)  # embedding-like
    x[5, :] = 0.0
    x[5, 0] = 1.0                                  # one-hot
    return x


def test_int8_filter_bound_holds_for_inner_product():
    rng = np.random.default_rng(11)
    d = 1536
    x = _rows(rng, 64, d)
    q = _rows(rng, 16, d)
    cx, sx, rx2 = _quantize_i8(x)
    cq, sq, rq2 = _quantize_i8(q)
    dot = (cq @ cx.T).astype(np.int64)
    assert np.abs(dot).max() < 2 ** 31
    f = (sq[:, None] * sx[None, :]).astype(np.float32)
    approx = (dot.astype(np.float32) * f).astype(np.float64)
    exact = q.astype(np.float64) @ x.astype(np.float64).T
    xn = np.linalg.norm(x.astype(np.float64), axis=1)
    qn = np.linalg.norm(q.astype(np.float64), axis=1)
    rx = np.sqrt(rx2.astype(np.float64))
    rq = np.sqrt(rq2.astype(np.float64))
    hx = xn + rx
    hq = qn + rq
    B = (_GAM_I8 * np.outer(hq, hx) + np.outer(rq, hx) + np.outer(hq, rx) + np.outer(rq, rx)
         + 2 * _U * np.outer(qn, xn)) * (1 + 1e-6)
    err = np.abs(approx - exact)
    assert (err <= B).all(), float((err - B).max())
    # the bound is not vacuous: for uniform rows it is a few per mille of |x||q|
    assert np.median(B[6:, 6:] / np.outer(qn[6:], xn[6:])) < 0.01


def test_int8_filter_bound_holds_for_cosine():
    rng = np.random.default_rng(12)
    d = 768
    x = _rows(rng, 80, d)
    # the cosine ranks no zero-norm rows (their inverse norm is infinite)
    x[1] = rng.uniform(-1, 1, d)
    x[2] = rng.uniform(-1, 1, d) * 1e-3
    cx, sx, rx2 = _quantize_i8(x)
    xn2 = (x.astype(np.float32) ** 2).sum(axis=1, dtype=np.float32)
    xinv = (1.0 / np.sqrt(xn2.astype(np.float64))).astype(np.float32)
    fx = (sx * xinv).astype(np.float32)                 # folded s / |x|
    dot = cx @ cx.T
    key_a = -((dot.astype(np.float32) * (fx[:, None] * fx[None, :]).astype(np.float32))
              .astype(np.float32)).astype(np.float64)
    ip = (x.astype(np.float64) @ x.astype(np.float64).T).astype(np.float32)
    key_e = -((ip * xinv[:, None]).astype(np.float32) * xinv[None, :]).astype(np.float64)
    rho = np.sqrt((rx2.astype(np.float64) / xn2.astype(np.float64)).max())
    gam_ld = (d + 1) * 2.0 ** -23 / (1 - (d + 1) * 2.0 ** -23)
    norm_inf = 2 * gam_ld
    rel = _GAM_I8 * (1 + rho) ** 2 + 2 * rho * (1 + rho) + rho ** 2 + 2.0 ** -23
    b = (rel * (1 + 1.5 * norm_inf) + 2.0 ** -22) * (1 + 1e-6)
    assert (np.abs(key_a - key_e) <= b).all(), float(np.abs(key_a - key_e).max() - b)


def _l2aug_params(x, xn):
    """vs_gemm_x1.hip l2aug_params: C = mean max|x| over the nonzero rows, nref
    = the largest norm, m = max |nref - n_x| / (2 C max|x|) rounded up to 64
    (at least 64)."""
    mx = np.abs(x).max(axis=1).astype(np.float64)
    on = mx > 0
    C = float(np.float32(mx[on].mean()))
    nref = float(np.float32(xn[on].max()))
    need = (np.abs(nref - xn[on].astype(np.float64)) / mx[on]).max() / (2.0 * C)
    return max(64, int(np.ceil(need / 64.0) * 64)), C, nref


def _quantize_i8_l2aug_rows(x, xn, m, C, nref):
    """quantize_i8_l2aug_kernel, rows: x' = [x, e], sum_j C e_j = (nref - n_x) / 2;
    the extra codes split T = rint(E / s) evenly; returns codes, s,
    |x'-p(x')|^2 and |x'|^2 (rounded up)."""
    x = np.asarray(x, np.float32)
    mx = np.abs(x).max(axis=1)
    E = (np.float64(nref) - xn.astype(np.float64)) / (2.0 * np.float64(C))
    sd = np.maximum(mx.astype(np.float64), np.abs(E) / m) / 127.0
    s = sd.astype(np.float32)
    s = np.where(s.astype(np.float64) < sd, np.nextafter(s, np.float32(np.inf)), s)
    with np.errstate(divide="ignore", invalid="ignore"):
        c = np.where(s[:, None] > 0, np.rint(x / s[:, None]), 0.0)
        T = np.where(s > 0, np.rint(E / s.astype(np.float64)), 0.0)
    c = np.clip(c, -127, 127).astype(np.int64)
    T = np.clip(T, -127.0 * m, 127.0 * m).astype(np.int64)
    base = np.trunc(T / m).astype(np.int64)
    rem = T - base * m
    j = np.arange(m)[None, :]
    ce = base[:, None] + np.where(j < np.abs(rem)[:, None], np.sign(rem)[:, None], 0)
    assert np.abs(ce).max() <= 127
    r = x.astype(np.float64) - s[:, None].astype(np.float64) * c
    dlt = np.abs(E - s.astype(np.float64) * T) + np.abs(E) * 1e-15
    rn2 = ((r * r).sum(axis=1) + dlt * dlt / m) * (1 + 1e-12)
    d1 = (E - s.astype(np.float64) * T) / m
    e = s[:, None].astype(np.float64) * ce + d1[:, None]        # the conceptual extra entries
    an2 = ((x.astype(np.float64) ** 2).sum(axis=1) + (e * e).sum(axis=1)) * (1 + 1e-12)
    return np.concatenate([c, ce], axis=1), s, rn2, an2


def _quantize_i8_l2aug_queries(q, m, C):
    q = np.asarray(q, np.float32)
    mx = np.abs(q).max(axis=1)
    C32 = np.float32(C)
    with np.errstate(divide="ignore"):
        cq = np.where(mx > C32, np.clip(np.floor(np.float32(127.0) * (C32 / mx)), 1, 127), 127)
    cq = cq.astype(np.int64)
    s = (C32 / cq.astype(np.float32)).astype(np.float32)
    c = np.clip(np.rint(q / s[:, None]), -127, 127).astype(np.int64)
    r = q.astype(np.float64) - s[:, None].astype(np.float64) * c
    re = np.float64(C32) - s.astype(np.float64) * cq
    rn2 = ((r * r).sum(axis=1) + m * re * re) * (1 + 1e-12)
    ce = np.repeat(cq[:, None], m, axis=1)
    return np.concatenate([c, ce], axis=1), s, rn2


def test_int8_l2_augmented_bound_holds():
    """L2 on the int8 plane (vs_gemm_x1.hip quantize_i8_l2aug_kernel, bound_key's
    l2aug branch, l2aug_map_kernel): the pass scores the augmented vectors
    x' = [x, e] (sum_j C e_j = (nref - n_x) / 2) and q' = [q, C ..] with the
    inner product's int8 arithmetic, A = -fl(fl(sum) fl(s_q s_x)) ~ n_x / 2 -
    q.x - nref / 2; the list keys become max(0, fl(fl(qn + nref) + 2A)) (the
    rows' extra entries stay small: their norms sit near nref); faiss's L2 key is
    max(0, fl(fl(qn + n_x) - fl(2 fl(q.x)))).  Every pair is within the bound,
    zero, tiny, outlier, embedding-like and one-hot rows included, and the bound
    is not vacuous on uniform rows."""
    rng = np.random.default_rng(21)
    d = 1536
    x = _rows(rng, 64, d)
    q = _rows(rng, 16, d)
    q[5] = -x[9]                                   # a query far from everything
    q[6] = x[10]                                   # a query equal to a row
    xn = (x.astype(np.float32) ** 2).sum(axis=1, dtype=np.float32)
    qn = (q.astype(np.float32) ** 2).sum(axis=1, dtype=np.float32)
    m, C, nref = _l2aug_params(x[6:], xn[6:])      # the uniform bulk sets them
    assert m == 64  # uniform rows' norms lie within a few per cent of each other
    cx, sx, rx2, ax2 = _quantize_i8_l2aug_rows(x, xn, m, C, nref)
    cq, sq, rq2 = _quantize_i8_l2aug_queries(q, m, C)
    dot = (cq @ cx.T).astype(np.int64)
    assert np.abs(dot).max() < 2 ** 31
    f = (sq[:, None] * sx[None, :]).astype(np.float32)
    A = -(dot.astype(np.float32) * f).astype(np.float32)
    qr = (qn + np.float32(nref)).astype(np.float32)
    Ahat = np.maximum(np.float32(0), (qr[:, None] + np.float32(2) * A).astype(np.float32))
    ip = (q.astype(np.float64) @ x.astype(np.float64).T).astype(np.float32)
    K = np.maximum(np.float32(0), ((qn[:, None] + xn[None, :]).astype(np.float32)
                                   - np.float32(2) * ip).astype(np.float32))
    # bound_key, l2aug: index maxima of |x'|^2 and |r(x')|^2, the query's own
    axm2, rxm2 = ax2.max(), rx2.max()
    hx = np.sqrt(axm2) + np.sqrt(rxm2)
    rx = np.sqrt(rxm2)
    qn64 = (q.astype(np.float64) ** 2).sum(axis=1)
    rq = np.sqrt(rq2)
    hq = np.sqrt(qn64 + m * np.float64(np.float32(C)) ** 2) + rq
    b = (_GAM_I8 * hx * hq + hx * rq + rx * hq + rx * rq) * (1 + 1e-6)
    B = (2 * b + 8 * _U * (qn.astype(np.float64) + axm2)
         + 2 * _U * (qn.astype(np.float64) + nref + 2.01 * hx * hq)) * (1 + 1e-6)
    err = np.abs(Ahat.astype(np.float64) - K.astype(np.float64))
    assert (err <= B[:, None]).all(), float((err - B[:, None]).max())
    # not vacuous: over an index of the uniform rows alone (the outlier row's
    # scale sets the maxima above), a small part of the L2 key spread
    axm2, rxm2 = ax2[6:].max(), rx2[6:].max()
    hx = np.sqrt(axm2) + np.sqrt(rxm2)
    rx = np.sqrt(rxm2)
    b = (_GAM_I8 * hx * hq + hx * rq + rx * hq + rx * rq) * (1 + 1e-6)
    B = (2 * b + 8 * _U * (qn.astype(np.float64) + axm2)
         + 2 * _U * (qn.astype(np.float64) + nref + 2.01 * hx * hq)) * (1 + 1e-6)
    assert (err[6:, 6:] <= B[6:, None]).all()
    spread = K[6:, 6:].astype(np.float64).std()
    assert np.median(B[6:]) < 0.25 * spread, (np.median(B[6:]), spread)


def _bf16(x):
    """Round-to-nearest-even bf16 (as float32 values)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) >> 16 << 16
    return u.astype(np.uint32).view(np.float32)


def test_bf16_l2_augmented_bound_holds():
    """The bf16 plane's form of L2 as an inner product (vs_gemm_x1.hip
    bf16_plane_l2aug_kernel): x' = [bf16(x), 64 x bf16(E / 64)], E = (nref -
    n_x) / (2 Cb), q' = [bf16(q), Cb ..] with Cb a power of two (exact); the
    MFMA accumulates the products in fp32 (any order: gamma(ld + 1)); the list
    key max(0, fl(fl(qn + nref) - 2 fl(sum))) is within the bound of faiss's
    L2 key for every pair."""
    rng = np.random.default_rng(22)
    d, m = 1536, 64
    x = _rows(rng, 48, d)
    q = _rows(rng, 12, d)
    q[6] = x[10]
    xn = (x.astype(np.float32) ** 2).sum(axis=1, dtype=np.float32)
    qn = (q.astype(np.float32) ** 2).sum(axis=1, dtype=np.float32)
    _, C, nref = _l2aug_params(x[6:], xn[6:])
    Cb = float(2.0 ** np.round(np.log2(C)))
    E = (np.float64(nref) - xn.astype(np.float64)) / (2 * Cb)
    es = _bf16((E / m).astype(np.float32)).astype(np.float64)
    d1 = (E - m * es) / m
    hx_rows = np.concatenate([_bf16(x), np.repeat(es[:, None], m, axis=1).astype(np.float32)], 1)
    hq_rows = np.concatenate([_bf16(q), np.full((q.shape[0], m), Cb, np.float32)], 1)
    r = x.astype(np.float64) - _bf16(x).astype(np.float64)
    rx2 = (r * r).sum(axis=1) + m * (np.abs(d1) + np.abs(E) * 1e-15 / m) ** 2
    ax2 = (x.astype(np.float64) ** 2).sum(axis=1) + m * (es + d1) ** 2
    # fp32 accumulation in row order (one of the orders the bound covers)
    prod = hq_rows.astype(np.float32)[:, None, :] * hx_rows.astype(np.float32)[None, :, :]
    s32 = np.zeros(prod.shape[:2], np.float32)
    for j in range(prod.shape[2]):
        s32 = (s32 + prod[:, :, j]).astype(np.float32)
    A = -s32
    qr = (qn + np.float32(nref)).astype(np.float32)
    Ahat = np.maximum(np.float32(0), (qr[:, None] + np.float32(2) * A).astype(np.float32))
    ip = (q.astype(np.float64) @ x.astype(np.float64).T).astype(np.float32)
    K = np.maximum(np.float32(0), ((qn[:, None] + xn[None, :]).astype(np.float32)
                                   - np.float32(2) * ip).astype(np.float32))
    n_ = d + m + 1
    gam = n_ * 2.0 ** -23 / (1 - n_ * 2.0 ** -23)
    qr_ = q.astype(np.float64) - _bf16(q).astype(np.float64)
    rq = np.sqrt((qr_ * qr_).sum(axis=1))
    hq = np.sqrt((_bf16(q).astype(np.float64) ** 2).sum(axis=1) + m * Cb * Cb)
    hx = np.sqrt(ax2.max()) + np.sqrt(rx2.max())
    rx = np.sqrt(rx2.max())
    b = (gam * hx * hq + hx * rq + rx * hq + rx * rq) * (1 + 1e-6)
    B = (2 * b + 8 * _U * (qn.astype(np.float64) + ax2.max())
         + 2 * _U * (qn.astype(np.float64) + nref + 2.01 * hx * hq)) * (1 + 1e-6)
    err = np.abs(Ahat.astype(np.float64) - K.astype(np.float64))
    assert (err <= B[:, None]).all(), float((err - B[:, None]).max())


def test_wide_threshold_below_the_floor_is_exact():
    """The wide check may use any T' <= T (vs_gemm_x1.hip verify_wide_kernel):
    with a_M the M-th smallest approximate key, T' = min(T, a_M + 2.000001 B)
    keeps every row outside S at key >= T' and the M best-approximate rows in S
    (exact keys <= a_M + B), so the check passes whenever T' < T; whenever it
    accepts, S holds the exact top-M.  Deep lists (many lists, far floors) shrink
    S to the rows near the top."""
    rng = np.random.default_rng(99)
    B, M = 1e-3, 19
    accepted = 0
    sizes = []
    for q in range(80):
        n = 4000
        e = rng.standard_normal(n)
        if q % 3:
            e[rng.choice(n, 60, replace=False)] = -5.0 + rng.uniform(0, 6 * B, 60)
        a = e + rng.uniform(-B, B, n)
        lists = _lane_lists(a, 128, 8, rng)
        full = [lst for lst in lists if len(lst) == 8]
        T = min(a[lst[-1]] for lst in full)
        entries = np.concatenate(lists)
        aM = np.sort(a[entries])[M - 1]
        Tp = min(T, aM + 2.000001 * B)
        S = [r for r in entries if a[r] < Tp]
        ok, top = _accept(S, Tp, e, B, M)
        if Tp < T:
            assert ok  # passes by construction when the threshold is below the floor
        if ok:
            accepted += 1
            sizes.append(len(S))
            exact = np.lexsort((np.arange(n), e))[:M]
            np.testing.assert_array_equal(top, exact)
    assert accepted == 80
    assert max(sizes) < 128 * 8


def test_wide_threshold_from_first_check_exact_keys():
    """The tighter wide threshold (verify_wide_kernel): e1_M, the M-th exact key
    among the first check's KF best-approximate rows, bounds the true E_M from
    above, so T' = min(T, a_M + 2.000001 B, e1_M + 1.000001 B) keeps every row
    outside S at an exact key > e1_M >= E_M; the M rows behind e1_M are in S.
    The check passes whenever T' < T, S holds the exact top-M, and S is about
    half the size the a_M + 2B window gives.  Errors here sit at the bound's
    edges (+-B) as well as inside it."""
    rng = np.random.default_rng(7)
    B, M, KF = 1e-3, 19, 32
    tight, loose = [], []
    for q in range(80):
        n = 4000
        e = rng.standard_normal(n) * 0.01
        err = rng.uniform(-B, B, n)
        edge = rng.random(n) < 0.3
        err[edge] = np.where(rng.random(edge.sum()) < 0.5, -B, B)
        a = e + err
        lists = _lane_lists(a, 128, 8, rng)
        full = [lst for lst in lists if len(lst) == 8]
        T = min(a[lst[-1]] for lst in full)
        entries = np.concatenate(lists)
        first = entries[np.lexsort((entries, a[entries]))[:KF]]
        aM = np.sort(a[entries])[M - 1]
        e1M = np.sort(e[first])[M - 1]
        Tp = min(T, aM + 2.000001 * B, e1M + 1.000001 * B)
        S = [r for r in entries if a[r] < Tp]
        ok, top = _accept(S, Tp, e, B, M)
        if Tp < T:
            assert ok
        assert ok
        exact = np.lexsort((np.arange(n), e))[:M]
        np.testing.assert_array_equal(top, exact)
        tight.append(len(S))
        loose.append(sum(1 for r in entries if a[r] < min(T, aM + 2.000001 * B)))
    assert np.mean(tight) < 0.75 * np.mean(loose)


def _stream_lists(a, owner, P, L, order, cut_at=None, B=None, M=None, late=0):
    """Lane lists fed row by row in `order` (admission key < the list's last
    entry, as the kernel's), optionally with a query cut set after the first
    `cut_at` rows: cut = a_M(lists now) + 2.000001 B, and later rows are admitted
    only below min(last, cut) (vs_gemm_x1.hip "Query cuts").  Returns the lists,
    the cut (inf without one) and the number of rows admitted after row
    `late` (= cut_at or the same point of the run without a cut)."""
    lists = [[] for _ in range(P)]
    cut = np.inf
    admitted = 0
    for i, r in enumerate(order):
        if cut_at is not None and i == cut_at:
            ent = np.array([a[x] for lst in lists for x in lst])
            if len(ent) >= M:
                cut = np.nextafter(np.float32(np.sort(ent)[M - 1] + 2.000001 * B),
                                   np.float32(np.inf))
        lst = lists[owner[r]]
        lim = a[lst[-1]] if len(lst) == L else np.inf
        if a[r] < min(lim, cut):
            admitted += i >= late
            lst.append(r)
            lst.sort(key=lambda x: (a[x], x))
            del lst[L:]
    return [np.array(lst, dtype=np.int64) for lst in lists], float(cut), admitted


def test_query_cut_keeps_both_checks_and_drops_admissions():
    """A cut a_M(snapshot) + 2.000001 B taken between two launches of the pass
    (the final a_M can only be lower) never changes what the checks decide: the
    wide threshold T' is the same (T' <= a_M + 2B <= cut), the rescored set is
    the same, the first check's outcome is the same; after the cut the lists
    admit a fraction of the rows they would."""
    rng = np.random.default_rng(5)
    B, M, KF, P, L = 1e-3, 19, 32, 128, 8
    fewer = []
    for q in range(40):
        n = 20000
        e = rng.standard_normal(n) * 0.01
        if q % 3 == 0:
            e[rng.choice(n, 50, replace=False)] = -0.05 + rng.uniform(0, 4 * B, 50)
        a = e + rng.uniform(-B, B, n)
        owner = rng.integers(0, P, size=n)
        order = rng.permutation(n)
        res = []
        for cut_at in (None, n // 8):
            lists, cut, admitted = _stream_lists(a, owner, P, L, order, cut_at, B, M, n // 8)
            full = [lst for lst in lists if len(lst) == L]
            T = min((a[lst[-1]] for lst in full), default=np.inf)
            T = min(T, cut)  # the verification's floor for the rows the cut dropped
            entries = np.concatenate(lists)
            srt = entries[np.lexsort((entries, a[entries]))]
            aM = a[srt[M - 1]]
            merged = srt[:KF]
            T1 = min(a[merged[-1]] if len(merged) == KF else np.inf, T)
            ok1, top1 = _accept(list(merged), T1, e, B, M)
            Tp = min(T, aM + 2.000001 * B)
            S = sorted(r for r in entries if a[r] < Tp)
            ok2, top2 = _accept(S, Tp, e, B, M)
            exact = np.lexsort((np.arange(n), e))[:M]
            for ok, top in ((ok1, top1), (ok2, top2)):
                if ok:
                    np.testing.assert_array_equal(top, exact)
            res.append((ok1, ok2, Tp, S, admitted, aM, cut))
        (o1, o2, tp0, s0, n0, am0, _), (c1, c2, tp1, s1, n1, am1, cut) = res
        assert am1 == am0 and cut >= am1 + 2 * B
        assert (o1, o2) == (c1, c2) and tp0 == tp1 and s0 == s1
        fewer.append(n1 / n0)
    assert np.mean(fewer) < 0.3


def _order_image(k):
    """vs_gemm_x1.hip key_order: float order as unsigned order."""
    u = np.asarray(k, np.float32).view(np.uint32).astype(np.uint64)
    return np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)


def _mth_smallest_by_bits(keys, valid, M):
    """qcut_kernel's selection restated: the largest x with fewer than M valid
    images below it, built bit by bit from the top (empty entries: image 2^32)."""
    img = np.where(valid, _order_image(keys), np.uint64(1 << 32))
    if int((img < (1 << 32)).sum()) < M:
        return None
    x = 0
    for b in range(31, -1, -1):
        if int((img < x + (1 << b)).sum()) < M:
            x += 1 << b
    u = np.uint32(x)
    back = np.uint32(u & 0x7FFFFFFF) if u & 0x80000000 else np.uint32(~u)
    return np.array([back], np.uint32).view(np.float32)[0]


def test_query_cut_selection_is_the_mth_smallest_key():
    rng = np.random.default_rng(3)
    for trial in range(200):
        n = int(rng.integers(1, 300))
        keys = (rng.standard_normal(n) * 10 ** rng.uniform(-3, 3)).astype(np.float32)
        if trial % 5 == 0:
            keys[: n // 2] = keys[0]                       # duplicates
        if trial % 7 == 0:
            keys[rng.random(n) < 0.2] = np.float32(-0.0)   # signed zeros
        valid = rng.random(n) < 0.9
        M = int(rng.integers(1, 40))
        got = _mth_smallest_by_bits(keys, valid, M)
        v = np.sort(keys[valid])
        if len(v) < M:
            assert got is None
        else:
            assert got == v[M - 1]  # -0.0 == 0.0: the order image ranks -0 first


def test_dump_and_replay_leave_the_lists_of_in_kernel_admission():
    """The dump launches (vs_gemm_x1.hip header) restated: after the first
    launch sets the cut, a lane stores one (row, raw sum) slot for every row
    of a block whose per-row test says it may be below the floor (a superset:
    the kernel's integer threshold comes from the launch's largest row factor,
    modelled here as a lower bound a_lo <= a of the row's key), in the order it
    meets them, and x1_replay admits the stored rows in that order against
    min(list last, cut).  The lists equal those of admitting every row
    in-kernel against min(list last, cut), and a list whose dumped rows exceed
    its R = 128 slots (x1_dump_slots) is reported (its query is then failed)."""
    rng = np.random.default_rng(11)
    B, M, P, L, R = 1e-3, 19, 64, 8, 128
    for trial in range(30):
        n = 16 * 2048
        a = (rng.standard_normal(n) * 0.01).astype(np.float64)
        if trial % 4 == 0:  # near-duplicates: many rows just above the top
            a[rng.choice(n, 400, replace=False)] = -0.04 + rng.uniform(0, B, 400)
        a_lo = a - np.abs(rng.standard_normal(n)) * 2e-3  # the per-row test's bound
        owner = np.repeat(rng.integers(0, P, size=n // 16), 16)  # blocks of 16 rows
        order = np.arange(n)
        cut_at = n // 8
        ref, cut, _ = _stream_lists(a, owner, P, L, order, cut_at, B, M, cut_at)
        # the first launch as a list launch, then dumps + replay
        first, _, _ = _stream_lists(a[:cut_at], owner[:cut_at], P, L, np.arange(cut_at),
                                    None, B, M, cut_at)
        lists = [list(lst) for lst in first]
        dumps = [[] for _ in range(P)]
        for b0 in range(cut_at, n, 16):
            blk = np.arange(b0, b0 + 16)
            if a_lo[blk].min() < cut:  # the block test: one maximum and a compare
                # one slot per row that clears the per-row threshold
                dumps[owner[b0]].extend(int(r) for r in blk if a_lo[r] < cut)
        overflow = [len(d) > R for d in dumps]
        assert any(len(d) > 0 for d in dumps)
        for p in range(P):
            if overflow[p]:
                continue
            lst = lists[p]
            for r in dumps[p]:
                lim = a[lst[-1]] if len(lst) == L else np.inf
                if a[r] < min(lim, cut):
                    lst.append(r)
                    lst.sort(key=lambda x: (a[x], x))
                    del lst[L:]
        for p in range(P):
            if not overflow[p]:
                np.testing.assert_array_equal(np.array(lists[p], dtype=np.int64), ref[p])
