"""CPU: the resident index service — wire protocol, request
coalescing, readers/writer ordering and error mapping.  The index is the
oracle-backed test double (tests/helpers.py); the same flows run on the GPU in
test_gpu_store.py::test_service_on_gpu."""

import threading

import numpy as np
import pytest

from helpers import OracleIndex
from oracle import flat
from vsearch import faiss as vfaiss
from vsearch import langchain as vlc
from vsearch.service import IndexService, RemoteFAISS
from vsearch.synth import SynthEmbeddings

KEY = b"test-secret"


@pytest.fixture
def store(monkeypatch):
    monkeypatch.setattr(vfaiss, "IndexFlatL2", lambda d, **kw: OracleIndex(d, flat.METRIC_L2))
    monkeypatch.setattr(vfaiss, "IndexFlatIP",
                        lambda d, **kw: OracleIndex(d, flat.METRIC_INNER_PRODUCT))
    emb = SynthEmbeddings(48)
    texts = [f"book {i}" for i in range(200)]
    metas = [{"book_id": f"B{i:03d}", "genre": ["fantasy", "mystery", "science"][i % 3]}
             for i in range(200)]
    return vlc.FAISS.from_texts(texts, emb, metadatas=metas)


def _same(a, b):
    assert [(d.page_content, d.metadata, d.id) for d, _ in a] == \
           [(d.page_content, d.metadata, d.id) for d, _ in b]
    assert [float(s) for _, s in a] == [float(s) for _, s in b]


def test_remote_reads_match_local(store):
    with IndexService(store, authkey=KEY) as svc, RemoteFAISS(svc.address, KEY) as cli:
        assert cli.index.ntotal == 200 and cli.index.d == 48
        assert cli.index.metric_type == flat.METRIC_L2
        for q in ["book 7", "space adventure", "friendship animals"]:
            _same(cli.similarity_search_with_score(q, k=5),
                  store.similarity_search_with_score(q, k=5))
        vec = store.embedding_function.embed_query("book 11")
        _same(cli.similarity_search_with_score_by_vector(vec, k=4, filter={"genre": "mystery"},
                                                         fetch_k=30),
              store.similarity_search_with_score_by_vector(vec, k=4, filter={"genre": "mystery"},
                                                           fetch_k=30))
        _same(cli.similarity_search_with_score("book 3", k=10, score_threshold=1.5),
              store.similarity_search_with_score("book 3", k=10, score_threshold=1.5))
        assert [d.id for d in cli.similarity_search("book 9", k=3)] == \
               [d.id for d in store.similarity_search("book 9", k=3)]
        xq = np.asarray([store.embedding_function.embed_query(f"q{i}") for i in range(7)],
                        dtype=np.float32)
        D, I = cli.index.search(xq, 6)
        Dl, Il = store.index.search(xq, 6)
        np.testing.assert_array_equal(I, Il)
        np.testing.assert_array_equal(D, Dl)
        np.testing.assert_array_equal(cli.index.reconstruct(5), store.index.reconstruct(5))


def test_concurrent_searches_coalesce_and_match(store):
    emb = store.embedding_function
    queries = [f"query {i}" for i in range(64)]
    want = {q: store.similarity_search_with_score(q, k=5) for q in queries}
    got = {}
    barrier = threading.Barrier(16, timeout=30)

    with IndexService(store, authkey=KEY) as svc:
        def worker(qs):
            with RemoteFAISS(svc.address, KEY) as cli:
                barrier.wait()
                for q in qs:
                    got[q] = cli.similarity_search_with_score(q, k=5)

        ts = [threading.Thread(target=worker, args=(queries[i::16],)) for i in range(16)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
        st = svc.stats
    for q in queries:
        _same(got[q], want[q])
    assert st["search_rows"] == 64
    assert st["search_batches"] <= 64  # coalescing never adds engine calls
    del emb


def test_slow_engine_requests_are_stacked(store):
    """While one engine call runs, the requests that arrive are stacked into the
    next call: 16 concurrent clients need fewer than 16 engine calls."""
    real = store.index.search
    calls = []

    def slow_search(x, k):
        calls.append(x.shape[0])
        threading.Event().wait(0.05)
        return real(x, k)

    store.index.search = slow_search
    queries = [f"q{i}" for i in range(16)]
    want = {q: store.similarity_search_with_score(q, k=3) for q in queries}
    calls.clear()
    got = {}
    with IndexService(store, authkey=KEY) as svc:
        barrier = threading.Barrier(16, timeout=30)

        def worker(q):
            with RemoteFAISS(svc.address, KEY) as cli:
                barrier.wait()
                got[q] = cli.similarity_search_with_score(q, k=3)

        ts = [threading.Thread(target=worker, args=(q,)) for q in queries]
        for t in ts:
            t.start()
        for t in ts:
            t.join(60)
    for q in queries:
        _same(got[q], want[q])
    assert sum(calls) == 16 and len(calls) < 16 and max(calls) > 1


def test_remote_writes_and_errors(store, tmp_path):
    with IndexService(store, authkey=KEY, save_root=str(tmp_path)) as svc, \
            RemoteFAISS(svc.address, KEY) as cli:
        ids = cli.add_texts(["new book"], metadatas=[{"book_id": "B999"}])
        assert cli.index.ntotal == 201 and store.index.ntotal == 201
        assert cli.get_by_ids(ids)[0].page_content == "new book"
        cli.upsert_texts(["new book v2"], metadatas=[{"book_id": "B999"}])
        assert cli.index.ntotal == 201
        assert cli.similarity_search("new book v2", k=1)[0].metadata["book_id"] == "B999"
        with pytest.raises(ValueError):
            cli.delete(["no-such-id"])
        with pytest.raises(ValueError):
            cli.add_texts(["a", "b"], ids=["dup", "dup"])
        with pytest.raises(AssertionError):
            cli.index.search(np.zeros((1, 7), np.float32), 3)
        with pytest.raises(ValueError):
            cli.similarity_search("x", filter=lambda m: True)
        assert cli.delete(ids=store.ids_for_key("B000")) is True
        assert cli.index.ntotal == 200
        cli.save_local("vs")
    assert (tmp_path / "vs" / "index.faiss").exists()


def test_save_confined_and_read_only(store, tmp_path):
    root = tmp_path / "root"
    root.mkdir()
    with IndexService(store, authkey=KEY) as svc, RemoteFAISS(svc.address, KEY) as cli:
        with pytest.raises(PermissionError):  # no save_root: save_local disabled
            cli.save_local("vs")
    with IndexService(store, authkey=KEY, save_root=str(root)) as svc, \
            RemoteFAISS(svc.address, KEY) as cli:
        for bad in (str(tmp_path / "elsewhere"), "../escape", "/etc"):
            with pytest.raises(PermissionError):
                cli.save_local(bad)
        with pytest.raises(PermissionError):
            cli.save_local("ok", index_name="../../x")
        cli.save_local("sub/ok")
        assert (root / "sub" / "ok" / "index.faiss").exists()
    assert not (tmp_path / "elsewhere").exists() and not (tmp_path / "escape").exists()
    with IndexService(store, authkey=KEY, read_only=True, save_root=str(root)) as svc, \
            RemoteFAISS(svc.address, KEY) as cli:
        assert cli.index.ntotal == 200
        for call in (lambda: cli.add_texts(["x"]), lambda: cli.delete(["a"]),
                     lambda: cli.upsert_texts(["x"], [{"book_id": "B1"}]),
                     lambda: cli.save_local("ro")):
            with pytest.raises(PermissionError):
                call()
        assert cli.index.ntotal == 200


def test_authkey_required(store):
    with pytest.raises(TypeError):
        IndexService(store)  # noqa: the key has no default
    with pytest.raises(ValueError):
        IndexService(store, authkey=b"")


def test_bad_authkey_rejected(store):
    with IndexService(store, authkey=b"right") as svc:
        with pytest.raises(Exception):
            RemoteFAISS(svc.address, authkey=b"wrong")
        with RemoteFAISS(svc.address, authkey=b"right") as cli:
            assert cli.index.ntotal == 200
