"""GPU: the drop-in store and the student self-join end to end on libvsearch,
reproducing the reference call sites on the CSV sample (BASELINE config 1)."""

import numpy as np
import pytest

from oracle import flat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def catalog_store(golden):
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, _ = golden
    # book_vector/main.py:469 full rebuild: FAISS.from_texts(texts, embeddings, metadatas=...)
    return vlc.FAISS.from_texts(inputs["book_texts"], SynthEmbeddings(),
                                metadatas=inputs["book_metadata"])


def test_search_catalog_flow(catalog_store, golden):
    """mcp_book_server.py:142-146: similarity_search(keyword, k) -> book_id + snippet[:200]."""
    inputs, exp = golden
    for qi, kw in enumerate(inputs["keywords"][:16]):
        docs = catalog_store.similarity_search(kw, k=5)
        results = [{"book_id": d.metadata["book_id"], "snippet": d.page_content[:200]} for d in docs]
        want = exp["books_l2_I"][341 + qi, :5]
        pos = {m["book_id"]: i for i, m in enumerate(inputs["book_metadata"])}
        assert [pos[r["book_id"]] for r in results] == want.tolist()
        assert all(len(r["snippet"]) <= 200 for r in results)


def test_scores_are_faiss_D(catalog_store, golden_vectors, golden):
    _, exp = golden
    _, xq, _ = golden_vectors
    res = catalog_store.similarity_search_with_score_by_vector(xq[400], k=10)
    D = np.array([s for _, s in res], dtype=np.float32)
    np.testing.assert_allclose(D, exp["books_l2_D"][400, :10], rtol=1e-5, atol=1e-5)


def test_delete_add_save_load(tmp_path, golden):
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, _ = golden
    emb = SynthEmbeddings()
    texts = inputs["book_texts"][:50]
    metas = inputs["book_metadata"][:50]
    ids = [m["book_id"] for m in metas]
    store = vlc.FAISS.from_texts(texts, emb, metadatas=metas, ids=ids)
    assert store.delete(["B002", "B010"])
    assert store.index.ntotal == 48
    assert "B002" not in store.index_to_docstore_id.values()
    store.add_texts([texts[1]], metadatas=[metas[1]], ids=["B002-v2"])
    assert store.index_to_docstore_id[48] == "B002-v2"
    top = store.similarity_search(texts[1], k=1)
    assert top[0].id == "B002-v2"
    store.save_local(str(tmp_path))
    loaded = vlc.FAISS.load_local(str(tmp_path), emb, allow_dangerous_deserialization=True)
    assert loaded.index.ntotal == 49
    np.testing.assert_array_equal(loaded.index.reconstruct_n(0, 49),
                                  store.index.reconstruct_n(0, 49))
    q = emb.embed_query("dragons and magic")
    a = [d.id for d in store.similarity_search_by_vector(q, k=7)]
    b = [d.id for d in loaded.similarity_search_by_vector(q, k=7)]
    assert a == b


def test_student_neighbours(golden, golden_vectors):
    from vsearch.students import pgvector_quantize, student_neighbours, student_neighbours_of

    inputs, _ = golden
    keys = inputs["student_keys"]
    _, _, xs = golden_vectors
    rows = student_neighbours(keys, xs, k=15, threshold=None)
    xq = pgvector_quantize(xs)
    S, I = flat.pgvector_cosine_topk(xq, 15)
    want = [(keys[a], keys[int(b)], float(S[a, j])) for a in range(25) for j, b in enumerate(I[a])
            if b >= 0]
    assert [(a, b) for a, b, _ in rows] == [(a, b) for a, b, _ in want]
    np.testing.assert_allclose([s for *_, s in rows], [s for *_, s in want], rtol=1e-5, atol=1e-6)
    # the refresher's threshold: random synthetic students are far below 0.75
    assert student_neighbours(keys, xs, k=15, threshold=0.75) == []
    one = student_neighbours_of(keys[3], keys, xs, k=15)
    assert one == [r for r in rows if r[0] == keys[3]]


def test_student_index_resident_events(golden, golden_vectors):
    """Per-event similarity on a resident StudentIndex: every event queries the
    kept index (no re-upload), equals the oracle, and a re-embedded student's
    row is replaced in place of a re-build."""
    from vsearch.students import StudentIndex, pgvector_quantize

    inputs, _ = golden
    keys = list(inputs["student_keys"])
    _, _, xs = golden_vectors
    si = StudentIndex(keys, xs)
    xq = pgvector_quantize(xs)
    S, I = flat.pgvector_cosine_topk(xq, 15)
    for a in (0, 3, 24):
        want = [(keys[a], keys[int(b)], float(S[a, j])) for j, b in enumerate(I[a]) if b >= 0]
        got = si.neighbours_of(keys[a], 15)
        assert [(x, y) for x, y, _ in got] == [(x, y) for x, y, _ in want]
        np.testing.assert_allclose([z for *_, z in got], [z for *_, z in want], rtol=1e-5,
                                   atol=1e-6)
    # student 5 re-embedded as a near copy of student 9: they become neighbours
    newv = xs[9] + 0.01 * xs[5]
    si.upsert(keys[5], newv)
    assert len(si) == 25 and si.index.ntotal == 25
    x2 = np.concatenate([np.delete(xs, 5, axis=0), newv[None, :]])
    keys2 = keys[:5] + keys[6:] + [keys[5]]
    S2, I2 = flat.pgvector_cosine_topk(pgvector_quantize(x2), 15)
    got = si.neighbours_of(keys[5], 15)
    assert got[0][1] == keys[9]
    assert [y for _, y, _ in got] == [keys2[int(b)] for b in I2[24] if b >= 0]


def test_sharded_single_rank_nccl():
    """The multi-GPU code path with world_size 1 over RCCL (merge kernel included)."""
    import os

    torch = pytest.importorskip("torch")
    import torch.distributed as dist

    from vsearch import faiss as vfaiss
    from vsearch.sharded import ShardedIndexFlat
    from vsearch.synth import synthetic_rows

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        idx = ShardedIndexFlat(64, vfaiss.METRIC_INNER_PRODUCT, device=0)
        idx.add_synthetic(20000, seed=3)
        xq = synthetic_rows(10**6, 40, 64, 4)
        D, I = idx.search(xq, 10)
        xb = synthetic_rows(0, 20000, 64, 3)
        Dr, Ir = flat.knn_exact(xb, xq, 10, vfaiss.METRIC_INNER_PRODUCT)
        assert not flat.mismatches(D, I, Dr, Ir, vfaiss.METRIC_INNER_PRODUCT, xb, xq)
        Dd, Id = idx.search_device(torch.from_numpy(xq).cuda(), 10,
                                   stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(Id.cpu().numpy(), I)
    finally:
        dist.destroy_process_group()


def test_upsert_on_gpu(golden):
    """§8 f4 delete-then-add on the HIP index: a re-embedded book keeps one row."""
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, _ = golden
    emb = SynthEmbeddings()
    texts, metas = inputs["book_texts"][:60], inputs["book_metadata"][:60]
    store = vlc.FAISS.from_texts(texts, emb, metadatas=metas)
    new = texts[7] + " (revised edition)"
    store.upsert_texts([new], metadatas=[metas[7]])
    assert store.index.ntotal == 60
    assert len(store.ids_for_key(metas[7]["book_id"])) == 1
    hit = store.similarity_search(new, k=1)[0]
    assert hit.page_content == new and hit.metadata["book_id"] == metas[7]["book_id"]
    want = np.stack([emb.embed_query(t) for t in texts[:7] + texts[8:] + [new]])
    np.testing.assert_array_equal(store.index.reconstruct_n(0, 60), want.astype(np.float32))


def test_service_on_gpu(catalog_store, golden):
    """§8 f2 resident service: concurrent remote searches, coalesced into shared
    engine calls on the HIP index, return the golden (oracle) book order and
    scores for every keyword — and what the in-process store returns."""
    import threading

    from vsearch.service import IndexService, RemoteFAISS

    inputs, exp = golden
    kws = inputs["keywords"][:32]
    pos = {m["book_id"]: i for i, m in enumerate(inputs["book_metadata"])}
    want = {kw: [(d.id, float(s)) for d, s in catalog_store.similarity_search_with_score(kw, k=5)]
            for kw in kws}
    got = {}
    key = b"gpu-test-secret"
    with IndexService(catalog_store, authkey=key) as svc:
        barrier = threading.Barrier(8, timeout=60)

        def worker(qs):
            with RemoteFAISS(svc.address, key) as cli:
                barrier.wait()
                for kw in qs:
                    got[kw] = [(d.id, float(s)) for d, s in cli.similarity_search_with_score(kw, k=5)]

        ts = [threading.Thread(target=worker, args=(kws[i::8],)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(90)
        assert svc.stats["search_rows"] == 32
    # a stacked batch may take faiss's other branch (nq >= 20: norm expansion,
    # SURVEY.md §8 a7), so scores agree to the fp32 tolerance, ids exactly
    for qi, kw in enumerate(kws):
        assert [i for i, _ in got[kw]] == [i for i, _ in want[kw]]
        np.testing.assert_allclose([s for _, s in got[kw]], [s for _, s in want[kw]],
                                   rtol=1e-5, atol=1e-5)
        # against the oracle's golden vectors (tests/golden/make_golden.py)
        ids = [catalog_store.docstore.search(i).metadata["book_id"] for i, _ in got[kw]]
        assert [pos[b] for b in ids] == exp["books_l2_I"][341 + qi, :5].tolist()
        np.testing.assert_allclose([s for _, s in got[kw]], exp["books_l2_D"][341 + qi, :5],
                                   rtol=1e-5, atol=1e-5)


def test_reference_store_migration_on_gpu(tmp_path, golden):
    """A reference-written directory (index.faiss + pickled index.pkl) is refused,
    rebuilt by full_faiss_rebuild on the HIP index, and reopened by load_local
    with the golden search order."""
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, exp = golden
    emb = SynthEmbeddings()
    d = tmp_path / "vector_store"
    d.mkdir()
    (d / "index.pkl").write_bytes(b"not loaded")
    (d / "index.faiss").write_bytes(b"IxF2")
    with pytest.raises(vlc.ReferenceStoreError):
        vlc.FAISS.load_local(str(d), emb, allow_dangerous_deserialization=True)
    vlc.full_faiss_rebuild(inputs["book_texts"], emb, inputs["book_metadata"], str(d))
    store = vlc.FAISS.load_local(str(d), emb, allow_dangerous_deserialization=True)
    assert store.index.ntotal == 341
    pos = {m["book_id"]: i for i, m in enumerate(inputs["book_metadata"])}
    for qi, kw in enumerate(inputs["keywords"][:8]):
        got = [pos[doc.metadata["book_id"]] for doc in store.similarity_search(kw, k=5)]
        assert got == exp["books_l2_I"][341 + qi, :5].tolist()


def test_reference_store_migration_without_reembedding_on_gpu(tmp_path, golden):
    """A faiss-written flat file (the reference's index.faiss, written here from
    the golden book embeddings with faiss's IxF2 layout) plus a pickle that is
    never read migrates to the HIP index with no embed_documents call, and the
    reopened store returns the golden search order."""
    from helpers import OracleIndex
    from vsearch import faiss as vfaiss
    from vsearch import langchain as vlc
    from vsearch.synth import SynthEmbeddings

    inputs, exp = golden
    emb = SynthEmbeddings()

    class NoEmbed:
        def embed_documents(self, t):
            raise AssertionError("the migration must not re-embed the catalogue")

        def embed_query(self, t):
            return emb.embed_query(t)

    d = tmp_path / "vector_store"
    d.mkdir()
    ref = OracleIndex(emb.dim, 1)
    ref.add(np.asarray(emb.embed_documents(inputs["book_texts"]), dtype=np.float32))
    vfaiss.write_index(ref, str(d / "index.faiss"))
    (d / "index.pkl").write_bytes(b"\x80\x04cos\nsystem\n.")
    with pytest.raises(vlc.ReferenceStoreError):
        vlc.FAISS.load_local(str(d), NoEmbed(), allow_dangerous_deserialization=True)
    vlc.migrate_reference_store(str(d), inputs["book_texts"], inputs["book_metadata"], NoEmbed(),
                                verify_sample=0)
    store = vlc.FAISS.load_local(str(d), NoEmbed(), allow_dangerous_deserialization=True)
    assert isinstance(store.index, vfaiss.IndexFlat) and store.index.ntotal == 341
    pos = {m["book_id"]: i for i, m in enumerate(inputs["book_metadata"])}
    for qi, kw in enumerate(inputs["keywords"][:8]):
        got = [pos[doc.metadata["book_id"]] for doc in store.similarity_search(kw, k=5)]
        assert got == exp["books_l2_I"][341 + qi, :5].tolist()
