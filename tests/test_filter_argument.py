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
