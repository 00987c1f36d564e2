"""CPU model of the paged exact engine's stopping rule (vs_support.hip
page_step_kernel / page_finish, vs_api.hip run_paged): a query's
lexicographic (key, label) order is read in pages of 64, and the next page is
fetched only while the page came back full and the answer needs more — fewer
than k entries so far, or (faiss's inner-product rule) the k-th key's run of
equal keys reaching the page's end below 2k - 1 entries.  The model checks
that the entries fetched that way always determine faiss's answer: the rule
applied to them (oracle/flat.py faiss_order, the restatement of
faiss_ip_tie_order) equals the rule applied to every row, on tie-heavy keys."""

import numpy as np
import pytest

from oracle import flat

PAGE = 64


def paged_entries(key, k, rule):
    """Entries (labels, keys) the engine accumulates for one query, in
    lexicographic order, following page_step's rule."""
    order = np.lexsort((np.arange(key.size), key))
    keys, labels = key[order], order
    need = 2 * k - 1 if rule else k
    npages = max(1, (min(need, key.size) + PAGE - 1) // PAGE)
    cnt = 0
    for p in range(npages):
        got = min(PAGE, key.size - cnt)
        cnt += got
        full = got == PAGE
        more = full and cnt < npages * PAGE and (
            cnt < k or (rule and cnt < 2 * k - 1 and keys[cnt - 1] == keys[k - 1]))
        if not more:
            break
    return labels[:cnt], keys[:cnt]


@pytest.mark.parametrize("levels", [3, 7, 40])
@pytest.mark.parametrize("k", [1, 5, 33, 64, 65, 100, 130, 300])
def test_pages_determine_faiss_rule(levels, k):
    rng = np.random.default_rng(levels * 1000 + k)
    for _ in range(20):
        n = int(rng.integers(1, 900))
        key = rng.integers(0, levels, n).astype(np.float32)  # long runs of ties
        for metric in (flat.METRIC_INNER_PRODUCT, flat.METRIC_L2):
            rule = metric == flat.METRIC_INNER_PRODUCT
            lab, kk = paged_entries(key, k, rule)
            got = flat.faiss_order(lab.astype(np.int64), kk, k, metric)
            want = flat.faiss_order(np.arange(n, dtype=np.int64), key, k, metric)
            np.testing.assert_array_equal(got, want)


def test_pages_stop_early_without_ties():
    """Distinct keys: ceil(k / 64) pages — one more only when the k-th entry
    ends a page (its run might go on) — never the 2k - 1 the rule could read."""
    key = np.random.default_rng(1).permutation(5000).astype(np.float32)
    for k in (10, 63, 64, 65, 100, 128, 2048):
        lab, _ = paged_entries(key, k, True)
        pages = -(-k // PAGE) + (1 if k % PAGE == 0 else 0)
        assert lab.size == pages * PAGE, (k, lab.size)
        lab, _ = paged_entries(key, k, False)  # L2 / raw: exactly ceil(k / 64)
        assert lab.size == -(-k // PAGE) * PAGE, (k, lab.size)
