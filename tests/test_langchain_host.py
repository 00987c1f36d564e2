"""CPU: host logic of the LangChain-compatible store and the faiss file format.

The arithmetic comes from an oracle-backed test double (tests/helpers.py) so the
docstore / label bookkeeping / argument checks / persistence can be exercised
without a GPU; the same flows run on the GPU in test_gpu_store.py."""

import os
import struct

import numpy as np
import pytest

from helpers import OracleIndex
from oracle import flat
from vsearch import faiss as vfaiss
from vsearch import langchain as vlc
from vsearch.synth import SynthEmbeddings, synth_embed


class StubEmbeddings:
    """The reference's own test stub (tests/test_integration_ingestion_graph.py:40-48)."""

    def embed_documents(self, texts, **_):
        return [[float(i % 3)] * 3 for i, _ in enumerate(texts)]

    def embed_query(self, text):
        return [0.0, 0.0, 0.0]


@pytest.fixture
def patched_indexes(monkeypatch):
    monkeypatch.setattr(vfaiss, "IndexFlatL2", lambda d, **kw: OracleIndex(d, flat.METRIC_L2))
    monkeypatch.setattr(vfaiss, "IndexFlatIP",
                        lambda d, **kw: OracleIndex(d, flat.METRIC_INNER_PRODUCT))


def test_from_texts_defaults_to_l2_and_stub_ranking(patched_indexes):
    texts = [f"book {i}" for i in range(10)]
    metas = [{"book_id": f"B{i:03d}"} for i in range(10)]
    store = vlc.FAISS.from_texts(texts, StubEmbeddings(), metadatas=metas)
    assert store.index.metric_type == flat.METRIC_L2
    assert store.distance_strategy == vlc.DistanceStrategy.EUCLIDEAN_DISTANCE
    assert store.index.ntotal == 10
    assert sorted(store.index_to_docstore_id) == list(range(10))
    docs = store.similarity_search("anything", k=4)
    # [i%3]*3 vs query 0: labels 0, 3, 6, 9 at distance 0 (lower label first)
    assert [d.metadata["book_id"] for d in docs] == ["B000", "B003", "B006", "B009"]
    res = store.similarity_search_with_score("anything", k=5)
    assert [float(s) for _, s in res] == [0.0, 0.0, 0.0, 0.0, 3.0]
    assert isinstance(res[0][1], np.floating)


def test_inner_product_strategy(patched_indexes):
    emb = SynthEmbeddings(32)
    texts = [f"t{i}" for i in range(20)]
    store = vlc.FAISS.from_texts(texts, emb, distance_strategy=vlc.DistanceStrategy.MAX_INNER_PRODUCT)
    assert store.index.metric_type == flat.METRIC_INNER_PRODUCT
    docs = store.similarity_search_with_score("t7", k=3)
    assert docs[0][0].page_content == "t7"
    assert abs(float(docs[0][1]) - 1.0) < 1e-5
    kept = store.similarity_search_with_score("t7", k=3, score_threshold=0.5)
    assert all(s >= 0.5 for _, s in kept)


def test_add_texts_ids_duplicates_and_lengths(patched_indexes):
    store = vlc.FAISS.from_texts(["a", "b"], SynthEmbeddings(8))
    ids = store.add_texts(["c", "d"], metadatas=[{"x": 1}, {"x": 2}], ids=["id-c", "id-d"])
    assert ids == ["id-c", "id-d"]
    assert store.index_to_docstore_id[2] == "id-c" and store.index_to_docstore_id[3] == "id-d"
    with pytest.raises(ValueError):
        store.add_texts(["e", "f"], ids=["dup", "dup"])
    with pytest.raises(ValueError):
        store.add_texts(["g"], metadatas=[{}, {}])
    with pytest.raises(ValueError):  # docstore rejects an existing id
        store.add_texts(["h"], ids=["id-c"])
    # re-embedding appends duplicates (book_vector/main.py:148): allowed with new ids
    store.add_texts(["c"])
    assert store.index.ntotal == 6 or store.index.ntotal == 7


def test_delete_renumbers_and_validates(patched_indexes):
    emb = SynthEmbeddings(16)
    texts = [f"doc{i}" for i in range(8)]
    ids = [f"id{i}" for i in range(8)]
    store = vlc.FAISS.from_texts(texts, emb, ids=ids)
    with pytest.raises(ValueError):
        store.delete(None)
    with pytest.raises(ValueError):
        store.delete(["nope"])
    assert store.delete(["id1", "id5"]) is True
    assert store.index.ntotal == 6
    assert store.index_to_docstore_id == {i: v for i, v in enumerate(
        ["id0", "id2", "id3", "id4", "id6", "id7"])}
    np.testing.assert_array_equal(store.index.reconstruct(1), synth_embed("doc2", 16))
    top = store.similarity_search("doc6", k=1)
    assert top[0].id == "id6"


def test_filter_and_fetch_k(patched_indexes):
    emb = SynthEmbeddings(16)
    texts = [f"doc{i}" for i in range(30)]
    metas = [{"genre": "a" if i % 2 else "b", "level": i} for i in range(30)]
    store = vlc.FAISS.from_texts(texts, emb, metadatas=metas)
    docs = store.similarity_search("doc3", k=3, filter={"genre": "a"}, fetch_k=30)
    assert len(docs) == 3 and all(d.metadata["genre"] == "a" for d in docs)
    assert docs[0].page_content == "doc3"
    docs = store.similarity_search("doc3", k=5, filter={"level": {"$gte": 20}}, fetch_k=30)
    assert all(d.metadata["level"] >= 20 for d in docs)
    docs = store.similarity_search("doc3", k=5, filter=lambda m: m["level"] < 3, fetch_k=30)
    assert {d.metadata["level"] for d in docs} <= {0, 1, 2}


def test_k_larger_than_store_skips_padding(patched_indexes):
    store = vlc.FAISS.from_texts(["x", "y"], SynthEmbeddings(8))
    assert len(store.similarity_search("x", k=10)) == 2


def test_reconstruct_weighted_query_flow(patched_indexes):
    """candidate_builder.py:166-168,184 — mean of reconstructed rated rows as the query."""
    emb = SynthEmbeddings(16)
    texts = [f"doc{i}" for i in range(12)]
    store = vlc.FAISS.from_texts(texts, emb, metadatas=[{"book_id": f"B{i}"} for i in range(12)])
    vecs = [store.index.reconstruct(i) for i in (2, 5)]
    q = np.mean(vecs, axis=0)
    ids = [d.metadata["book_id"] for d in store.similarity_search_by_vector(q, k=2)]
    assert set(ids) == {"B2", "B5"}


def test_save_load_roundtrip(tmp_path, patched_indexes):
    emb = SynthEmbeddings(8)
    store = vlc.FAISS.from_texts([f"t{i}" for i in range(5)], emb,
                                 metadatas=[{"book_id": i} for i in range(5)])
    store.save_local(str(tmp_path))
    assert (tmp_path / "index.faiss").exists() and (tmp_path / "index.docstore.json").exists()
    with pytest.raises(ValueError):
        vlc.FAISS.load_local(str(tmp_path), emb)
    loaded = vlc.FAISS.load_local(str(tmp_path), emb, allow_dangerous_deserialization=True,
                                  index_factory=lambda d, m: OracleIndex(d, m))
    assert loaded.index.ntotal == 5
    assert loaded.index_to_docstore_id == store.index_to_docstore_id
    np.testing.assert_array_equal(loaded.index.reconstruct_n(0, 5), store.index.reconstruct_n(0, 5))
    assert loaded.similarity_search("t3", k=1)[0].metadata["book_id"] == 3


def test_reference_written_store_migrates_by_full_rebuild(tmp_path, patched_indexes, golden):
    """A directory as the reference leaves it (index.faiss + LangChain's pickled
    index.pkl, book_vector/main.py:151,470): load_local refuses it without ever
    unpickling; the reference's own full rebuild (main.py:428-471) run through
    the drop-in rewrites it, and the rebuilt directory reopens with the same
    rows, labels and search results."""
    inputs, _ = golden
    emb = SynthEmbeddings(32)
    texts, metas = inputs["book_texts"][:40], inputs["book_metadata"][:40]
    ref_dir = tmp_path / "vector_store"
    ref_dir.mkdir()
    idx = OracleIndex(32, flat.METRIC_L2)
    idx.add(np.asarray(emb.embed_documents(texts), dtype=np.float32))
    vfaiss.write_index(idx, str(ref_dir / "index.faiss"))
    poison = b"\x80\x04cos\nsystem\n."  # a pickle that must never be loaded
    (ref_dir / "index.pkl").write_bytes(poison)
    with pytest.raises(vlc.ReferenceStoreError):
        vlc.FAISS.load_local(str(ref_dir), emb, allow_dangerous_deserialization=True,
                             index_factory=lambda d, m: OracleIndex(d, m))
    built = vlc.full_faiss_rebuild(texts, emb, metas, str(ref_dir))
    assert (ref_dir / "index.pkl").read_bytes() == poison  # untouched, not read
    loaded = vlc.FAISS.load_local(str(ref_dir), emb, allow_dangerous_deserialization=True,
                                  index_factory=lambda d, m: OracleIndex(d, m))
    assert loaded.index.ntotal == 40
    np.testing.assert_array_equal(loaded.index.reconstruct_n(0, 40), idx.reconstruct_n(0, 40))
    assert loaded.index_to_docstore_id == built.index_to_docstore_id
    for kw in inputs["keywords"][:5]:
        a = [(d.id, d.metadata["book_id"]) for d in built.similarity_search(kw, k=5)]
        b = [(d.id, d.metadata["book_id"]) for d in loaded.similarity_search(kw, k=5)]
        assert a == b


def test_reference_store_migrates_without_reembedding(tmp_path, patched_indexes, golden):
    """A reference-written directory (index.faiss + pickled index.pkl) migrates
    with the vectors of index.faiss kept and the docstore rebuilt from the
    catalogue rows in label order: no embed_documents call (beyond the optional
    sample check), the pickle never read, and the reopened store searches like
    the one the reference built."""
    inputs, _ = golden
    emb = SynthEmbeddings(32)
    texts, metas = inputs["book_texts"][:40], inputs["book_metadata"][:40]
    ref_dir = tmp_path / "vector_store"
    ref_dir.mkdir()
    idx = OracleIndex(32, flat.METRIC_L2)
    idx.add(np.asarray(emb.embed_documents(texts), dtype=np.float32))
    vfaiss.write_index(idx, str(ref_dir / "index.faiss"))
    poison = b"\x80\x04cos\nsystem\n."  # a pickle that must never be loaded
    (ref_dir / "index.pkl").write_bytes(poison)

    class Counting:
        def __init__(self):
            self.calls = 0

        def embed_documents(self, t):
            self.calls += len(t)
            return emb.embed_documents(t)

        def embed_query(self, t):
            return emb.embed_query(t)

    counting = Counting()
    factory = lambda d, m: OracleIndex(d, m)  # noqa: E731
    with pytest.raises(ValueError):  # a row count that is not the store's
        vlc.migrate_reference_store(str(ref_dir), texts[:39], metas[:39], counting,
                                    index_factory=factory)
    with pytest.raises(ValueError):  # rows out of label order fail the sample check
        vlc.migrate_reference_store(str(ref_dir), texts[::-1], metas[::-1], counting,
                                    verify_sample=3, index_factory=factory)
    with pytest.raises(ValueError):  # the order check is on by default
        vlc.migrate_reference_store(str(ref_dir), texts[1:] + texts[:1], metas[1:] + metas[:1],
                                    counting, index_factory=factory)
    with pytest.raises(ValueError):  # and needs embeddings unless switched off
        vlc.migrate_reference_store(str(ref_dir), texts, metas, None, index_factory=factory)

    class Noisy(Counting):  # a remote API: the same text, not the same bits
        def embed_documents(self, t):
            self.calls += len(t)
            e = np.asarray(emb.embed_documents(t), dtype=np.float64)
            return (e * (1 + 1e-4 * np.cos(np.arange(e.shape[1])))).tolist()

    noisy = Noisy()
    vlc.migrate_reference_store(str(ref_dir), texts, metas, noisy, index_factory=factory)
    assert noisy.calls == 8  # the default sample
    counting.calls = 0
    mig = vlc.migrate_reference_store(str(ref_dir), texts, metas, counting, verify_sample=4,
                                      index_factory=factory)
    assert counting.calls == 4  # the sample only: the catalogue is not re-embedded
    assert (ref_dir / "index.pkl").read_bytes() == poison
    loaded = vlc.FAISS.load_local(str(ref_dir), counting, allow_dangerous_deserialization=True,
                                  index_factory=factory)
    assert loaded.index.ntotal == 40
    np.testing.assert_array_equal(loaded.index.reconstruct_n(0, 40), idx.reconstruct_n(0, 40))
    assert loaded.index_to_docstore_id == mig.index_to_docstore_id
    assert [loaded.docstore.search(loaded.index_to_docstore_id[i]).metadata["book_id"]
            for i in range(40)] == [m["book_id"] for m in metas]
    ref = vlc.FAISS.from_texts(texts, emb, metadatas=metas)
    for kw in inputs["keywords"][:5]:
        a = [d.metadata["book_id"] for d in ref.similarity_search(kw, k=5)]
        b = [d.metadata["book_id"] for d in loaded.similarity_search(kw, k=5)]
        assert a == b


def test_faiss_flat_file_layout(tmp_path):
    idx = OracleIndex(3, flat.METRIC_INNER_PRODUCT)
    x = np.arange(12, dtype=np.float32).reshape(4, 3)
    idx.add(x)
    fn = tmp_path / "i.faiss"
    vfaiss.write_index(idx, str(fn))
    raw = fn.read_bytes()
    assert raw[:4] == b"IxFI"
    d, ntotal, d1, d2, trained, metric = struct.unpack("<iqqq?i", raw[4:37])
    assert (d, ntotal, d1, d2, trained, metric) == (3, 4, 1 << 20, 1 << 20, True, 0)
    (size,) = struct.unpack("<Q", raw[37:45])
    assert size == 12
    np.testing.assert_array_equal(np.frombuffer(raw[45:], dtype="<f4").reshape(4, 3), x)
    back = vfaiss.read_index(str(fn), index_factory=lambda d, m: OracleIndex(d, m))
    assert back.metric_type == 0
    np.testing.assert_array_equal(back.reconstruct_n(0, 4), x)
    bad = tmp_path / "bad.faiss"
    bad.write_bytes(b"IwFl" + raw[4:])
    with pytest.raises(RuntimeError):
        vfaiss.read_index(str(bad), index_factory=lambda d, m: OracleIndex(d, m))


def test_normalize_L2():
    x = np.array([[3.0, 4.0], [0.0, 0.0]], dtype=np.float32)
    vfaiss.normalize_L2(x)
    np.testing.assert_allclose(x[0], [0.6, 0.8], rtol=1e-6)
    assert (x[1] == 0).all()
    with pytest.raises(TypeError):
        vfaiss.normalize_L2(np.ones((2, 2), dtype=np.float64))


def test_docstore_semantics():
    ds = vlc.InMemoryDocstore()
    ds.add({"a": vlc.Document("x")})
    with pytest.raises(ValueError):
        ds.add({"a": vlc.Document("y")})
    assert ds.search("zz") == "ID zz not found."
    with pytest.raises(ValueError):
        ds.delete(["zz"])
    ds.delete(["a"])
    assert ds.search("a") == "ID a not found."


def test_pgvector_quantize_matches_text_roundtrip():
    from vsearch.students import pgvector_quantize

    rng = np.random.default_rng(0)
    v = rng.standard_normal((3, 50)).astype(np.float32) / 7
    q = pgvector_quantize(v)
    ref = np.array([[np.float32(float(f"{x:.6f}")) for x in row] for row in v], dtype=np.float32)
    np.testing.assert_array_equal(q, ref)


def test_synth_embed_deterministic_unit_norm():
    a = synth_embed("space adventure")
    b = synth_embed("space adventure")
    np.testing.assert_array_equal(a, b)
    assert a.dtype == np.float32 and a.shape == (1536,)
    assert abs(float(np.dot(a.astype(np.float64), a.astype(np.float64))) - 1.0) < 1e-6
    assert not np.array_equal(a, synth_embed("space adventures"))


def test_synthetic_rows_generator():
    from vsearch.synth import synthetic_rows

    x = synthetic_rows(5, 3, 7, seed=1234)
    assert x.dtype == np.float32 and x.shape == (3, 7)
    assert (x >= -1).all() and (x < 1).all()
    # scalar restatement of splitmix64 for one element
    M = (1 << 64) - 1

    def sm(z):
        z = (z + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)

    i, j = 6, 4
    z = sm(1234 ^ (i * 7 + j))
    assert x[1, 4] == np.float32((z >> 40) * 2.0 ** -23 - 1.0)
    np.testing.assert_array_equal(synthetic_rows(0, 10, 7, 1234)[5:8], x)


def test_upsert_replaces_reembedded_rows(patched_indexes):
    """a re-embedded book replaces its row instead of appending a
    duplicate (the reference appends: book_vector/main.py:148)."""
    emb = SynthEmbeddings(32)
    texts = [f"book {i}" for i in range(6)]
    metas = [{"book_id": f"B{i}"} for i in range(6)]
    store = vlc.FAISS.from_texts(texts, emb, metadatas=metas,
                                 distance_strategy=vlc.DistanceStrategy.MAX_INNER_PRODUCT)
    assert store.ids_for_key("B2") == [store.index_to_docstore_id[2]]
    # plain add_texts keeps the reference's append-duplicates behaviour
    store.add_texts(["book 2 v2"], metadatas=[{"book_id": "B2"}])
    assert store.index.ntotal == 7 and len(store.ids_for_key("B2")) == 2
    # upsert: both B2 rows go, one new row; B4 appears twice in the batch, last wins
    new_ids = store.upsert_texts(["book 2 v3", "book 4 v2", "book 4 v3", "fresh"],
                                 metadatas=[{"book_id": "B2"}, {"book_id": "B4"},
                                            {"book_id": "B4"}, {"book_id": "B9"}])
    assert len(new_ids) == 3
    assert store.index.ntotal == 6 - 2 + 3
    assert sorted(store.index_to_docstore_id) == list(range(store.index.ntotal))
    books = [store.docstore.search(store.index_to_docstore_id[i]).metadata["book_id"]
             for i in range(store.index.ntotal)]
    assert sorted(books) == ["B0", "B1", "B2", "B3", "B4", "B5", "B9"]
    assert books.count("B2") == 1 and books.count("B4") == 1
    # the index rows are the new embeddings, in label order
    want = np.array(emb.embed_documents(["book 0", "book 1", "book 3", "book 5", "book 2 v3",
                                         "book 4 v3", "fresh"]), dtype=np.float32)
    np.testing.assert_array_equal(store.index.reconstruct_n(0, store.index.ntotal), want)
    hit = store.similarity_search("book 4 v3", k=1)[0]
    assert hit.metadata["book_id"] == "B4" and hit.page_content == "book 4 v3"
    assert store.similarity_search("book 4 v2", k=1)[0].page_content != "book 4 v2"
    # the key map follows deletes
    store.delete(store.ids_for_key("B0"))
    assert store.ids_for_key("B0") == [] and store.index.ntotal == 6


def test_upsert_validates_before_mutating(patched_indexes):
    emb = SynthEmbeddings(16)
    store = vlc.FAISS.from_texts(["a", "b"], emb, metadatas=[{"book_id": 1}, {"book_id": 2}],
                                 ids=["ia", "ib"])
    with pytest.raises(ValueError):
        store.upsert_texts(["c"], metadatas=[{"book_id": 3}], ids=["ia"])  # id clash
    with pytest.raises(ValueError):
        store.upsert_texts(["c", "d"], metadatas=[{"book_id": 3}])  # length mismatch
    assert store.index.ntotal == 2
    # re-using the replaced row's own id is allowed (it is deleted first)
    store.upsert_texts(["a2"], metadatas=[{"book_id": 1}], ids=["ia"])
    assert store.index.ntotal == 2 and store.docstore.search("ia").page_content == "a2"
