"""GPU, BASELINE config C5 at scale: a bf16-stored corpus with interleaved
incremental remove / append and queries, through the multi-GPU front end
(ShardedIndexFlat, world 1 over gloo), in bench.py run_c5's pattern.

* 5M x 1536 bf16 rows (C5 is 50M: the same code path at a tenth of the rows,
  so the chunked fp64 oracle below finishes inside the test budget);
* three rounds of 1 % remove_ids (random labels, rng seed 91011) + 1 % append
  (new generator rows at the end of the label space), each followed by a
  batch-8 search (C5's batch);
* after each round: the label space is faiss's (stable compaction + append):
  sampled labels reconstruct to the generator rows the bookkeeping expects;
  the sampled queries are checked against a chunked fp64 oracle over the rows
  AS STORED (bf16-rounded rows and queries; reconstruct_n is bit-exact): every
  label among the proven candidates, labels exact except ties, scores within
  the fp32 contract (the bf16 engines accumulate in fp32);
* at the end: recall@10 of 1,000 queries against fp32 exact search over the
  same mutated corpus (fp32 indexes of the generator rows), >= 0.99.
Reference semantics: LangChain FAISS.delete -> faiss IndexFlat::remove_ids
(SURVEY.md §0.4 / Appendix A), appends as book_vector/main.py:148."""

import socket

import numpy as np
import pytest

from helpers import assert_against_candidates, oracle_merge, proven_candidates
from oracle import flat

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

N, D_, K, B = 5_000_000, 1536, 10, 8
ROUNDS = 3
SAMPLE = [0, 3, 7]


@pytest.fixture(scope="module")
def dist1():
    import torch.distributed as dist

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    yield dist
    dist.destroy_process_group()


def test_c5_interleaved_mutations_against_oracle(dist1):
    from vsearch import _lib
    from vsearch import faiss as vfaiss
    from vsearch.sharded import ShardedIndexFlat
    from vsearch.synth import synthetic_rows

    assert _lib.device_count() >= 1
    metric = flat.METRIC_INNER_PRODUCT
    index = ShardedIndexFlat(D_, metric, device=0, dtype="bf16")
    index.add_synthetic(N, seed=1234)
    assert index.ntotal == N and index.shard.dtype == "bf16"
    gen = np.arange(N, dtype=np.int64)  # generator row of every current label
    next_gen = N
    rng = np.random.default_rng(91011)
    nmut = N // 100
    xq_all = synthetic_rows(50_000_000, 1000 + ROUNDS * B, D_, 5678)
    for rnd in range(ROUNDS):
        rm = np.sort(rng.choice(gen.size, nmut, replace=False)).astype(np.int64)
        assert index.remove_ids(rm) == nmut
        gen = np.delete(gen, rm)
        add = np.arange(next_gen, next_gen + nmut, dtype=np.int64)
        next_gen += nmut
        index.append_synthetic_ids(add, seed=1234)
        gen = np.concatenate([gen, add])
        assert index.ntotal == gen.size == N
        # the label space: stable compaction, appends at the end
        probe = np.concatenate([rng.choice(N - nmut, 6, replace=False), [0, N - nmut - 1, N - nmut,
                                                                           N - 1]])
        for lab in probe:
            np.testing.assert_array_equal(
                index.shard.reconstruct(int(lab)),
                flat.round_bf16(synthetic_rows(int(gen[lab]), 1, D_, 1234)).ravel())
        xq = xq_all[1000 + rnd * B:1000 + (rnd + 1) * B]
        D, I = index.search(xq, K)
        assert D.shape == (B, K) and (I >= 0).all() and (I < N).all()
        assert (np.diff(D, axis=1) <= 0).all()
        rq = flat.round_bf16(xq[SAMPLE])
        cand = proven_candidates(index.shard, rq, metric, N, K)
        for row, q in enumerate(SAMPLE):
            assert_against_candidates(D[q], I[q], cand[row], metric, K, D_, strict=False)

    # recall@10 against fp32 exact search over the same (mutated) corpus
    nr = 1000
    xr = xq_all[:nr]
    _, Ib = index.search(xr, K)
    chunk = 2_500_000
    parts_D, parts_I = [], []
    for a in range(0, gen.size, chunk):
        ref = vfaiss.IndexFlat(D_, metric, device=0)
        ref.reserve(min(chunk, gen.size - a))
        ref.add_synthetic_ids(gen[a:a + chunk], seed=1234)
        ref.set_id_base(a)
        Dr, Ir = ref.search(xr, K, raw=True)
        parts_D.append(Dr)
        parts_I.append(Ir)
        del ref
    _, Im = oracle_merge(np.stack(parts_D), np.stack(parts_I), metric, K)
    recall = float(np.mean([len(set(Ib[i]) & set(Im[i])) / K for i in range(nr)]))
    print(f"C5 (5M rows, {ROUNDS} mutation rounds): recall@10 vs fp32 exact = {recall:.4f}")
    assert recall >= 0.99, recall


def test_c5_full_size_sampled_against_oracle(dist1):
    """C5 at its own size: 50M x 1536 bf16 rows, one round of 1 % removals and
    1 % appends, a batch-8 search; three sampled queries checked against the
    chunked fp64 oracle over all 50M rows as stored (proven candidate sets;
    reconstruct_n is bit-exact), so the full-size bf16 path has CPU-oracle
    parity and not only the bench's recall."""
    from vsearch.sharded import ShardedIndexFlat
    from vsearch.synth import synthetic_rows

    n = 50_000_000
    metric = flat.METRIC_INNER_PRODUCT
    index = ShardedIndexFlat(D_, metric, device=0, dtype="bf16")
    index.add_synthetic(n, seed=1234)
    rng = np.random.default_rng(4242)
    nmut = n // 100
    rm = np.sort(rng.choice(n, nmut, replace=False)).astype(np.int64)
    assert index.remove_ids(rm) == nmut
    index.append_synthetic_ids(np.arange(n, n + nmut, dtype=np.int64), seed=1234)
    assert index.ntotal == n
    xq = synthetic_rows(50_000_000, B, D_, 9876)
    D, I = index.search(xq, K)
    assert (I >= 0).all() and (I < n).all()
    rq = flat.round_bf16(xq[SAMPLE])
    cand = proven_candidates(index.shard, rq, metric, n, K, chunk=2_000_000)
    for row, q in enumerate(SAMPLE):
        assert_against_candidates(D[q], I[q], cand[row], metric, K, D_, strict=False)
    del index
