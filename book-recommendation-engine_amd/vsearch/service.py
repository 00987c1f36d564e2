"""Resident index service.

The reference reloads the whole store for every request: the recommendation
API spawns the MCP server as a subprocess per request (recommendation_api/
service.py:1739) and each tool call runs ``FAISS.load_local`` again
(mcp_book_server.py:64-66; candidate_builder.py:76-78).  At C3 scale that is a
61 GB read per query.  Here one long-lived process keeps the index resident in
HBM and serves the same vector-store calls to any number of clients:

* ``IndexService(store)`` serves a ``vsearch.langchain.FAISS`` store on a TCP
  socket (``multiprocessing.connection`` with an HMAC auth key).
* Concurrent searches are **coalesced**: requests that arrive while the engine
  is busy are stacked into one (B x d) batch and run as ONE ``index.search``
  (the skinny / GEMM engines instead of B separate GEMV scans), then split back.
  Each row's answer is what faiss returns for that row inside a batch of the
  stacked size: the same exact top-k; only the score's last bits can differ
  from a lone search, as faiss's own nq < 20 / nq >= 20 branches do (L2 direct
  sum vs norm expansion), within the fp32 tolerance.
* Writers (``add_texts`` / ``upsert_texts`` / ``delete`` / ``save_local``) take the
  store exclusively; readers share it (readers-writer lock), the same ordering
  faiss gives (concurrent ``search`` allowed, ``add`` exclusive).
* ``RemoteFAISS(address, authkey)`` is the client: the LangChain ``FAISS`` read /
  write surface the reference's call sites use, plus ``.index.ntotal/.d/.search``.
* Access: the HMAC auth key has no default (the caller supplies a secret);
  ``read_only=True`` refuses every write op; ``save_local`` writes only inside
  the ``save_root`` directory fixed when the server starts (refused when no
  root was given), never at an arbitrary client-chosen path.

Wire format: every message is one ``send_bytes`` frame = u32 header length +
UTF-8 JSON header + raw little-endian payload (float32 vectors, int64 labels).
Nothing is pickled in either direction.
"""

from __future__ import annotations

import argparse
import json
import logging
import os
import struct
import threading
from multiprocessing.connection import Client, Listener
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .langchain import FAISS, Document, _create_filter_func

logger = logging.getLogger(__name__)

__all__ = ["IndexService", "RemoteFAISS", "serve"]

_ERRORS = {"ValueError": ValueError, "AssertionError": AssertionError, "KeyError": KeyError,
           "TypeError": TypeError, "PermissionError": PermissionError}
_WRITE_OPS = ("add_texts", "upsert_texts", "delete", "save_local")


def _check_authkey(authkey) -> bytes:
    if not isinstance(authkey, (bytes, bytearray)) or len(authkey) == 0:
        raise ValueError("authkey: a non-empty bytes secret is required (no default)")
    return bytes(authkey)


def _pack(header: dict, payload: bytes = b"") -> bytes:
    h = json.dumps(header).encode("utf-8")
    return struct.pack("<I", len(h)) + h + payload


def _unpack(frame: bytes) -> Tuple[dict, memoryview]:
    (n,) = struct.unpack_from("<I", frame, 0)
    return json.loads(bytes(frame[4:4 + n]).decode("utf-8")), memoryview(frame)[4 + n:]


class _RWLock:
    """Readers share, a writer is exclusive; waiting writers block new readers."""

    def __init__(self):
        self._cv = threading.Condition()
        self._readers = 0
        self._writer = False
        self._waiting_writers = 0

    def acquire_read(self):
        with self._cv:
            while self._writer or self._waiting_writers:
                self._cv.wait()
            self._readers += 1

    def release_read(self):
        with self._cv:
            self._readers -= 1
            if not self._readers:
                self._cv.notify_all()

    def acquire_write(self):
        with self._cv:
            self._waiting_writers += 1
            while self._writer or self._readers:
                self._cv.wait()
            self._waiting_writers -= 1
            self._writer = True

    def release_write(self):
        with self._cv:
            self._writer = False
            self._cv.notify_all()


class _Pending:
    __slots__ = ("vec", "k", "done", "D", "I", "err")

    def __init__(self, vec: np.ndarray, k: int):
        self.vec, self.k = vec, k
        self.done = threading.Event()
        self.D = self.I = self.err = None


class _Coalescer:
    """Stacks concurrent single-query searches into one engine call.

    One dispatcher thread: it takes everything queued (up to max_batch rows),
    groups by k, runs one ``index.search`` per group, and hands each caller its
    rows.  Callers hold the service's read lock while they wait.  A lone
    request runs at once (no added wait)."""

    def __init__(self, service: "IndexService", max_batch: int):
        self._svc = service
        self._max_batch = max_batch
        self._cv = threading.Condition()
        self._queue: List[_Pending] = []
        self._stop = False
        self.batches = 0
        self.rows = 0
        self._thread = threading.Thread(target=self._run, name="vsearch-coalescer", daemon=True)
        self._thread.start()

    def submit(self, vec: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        p = _Pending(vec, k)
        with self._cv:
            self._queue.append(p)
            self._cv.notify()
        p.done.wait()
        if p.err is not None:
            raise p.err
        return p.D, p.I

    def stop(self):
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout=10)

    def _run(self):
        while True:
            with self._cv:
                while not self._queue and not self._stop:
                    self._cv.wait()
                if self._stop and not self._queue:
                    return
                take, rows = [], 0
                while self._queue and rows + self._queue[0].vec.shape[0] <= self._max_batch:
                    p = self._queue.pop(0)
                    take.append(p)
                    rows += p.vec.shape[0]
                if not take:  # one oversized request: run it alone
                    take = [self._queue.pop(0)]
            groups: Dict[int, List[_Pending]] = {}
            for p in take:
                groups.setdefault(p.k, []).append(p)
            for k, ps in groups.items():
                try:
                    x = np.concatenate([p.vec for p in ps]) if len(ps) > 1 else ps[0].vec
                    # every submitter holds the read lock while it waits, so no
                    # writer can run during this call
                    D, I = self._svc.store.index.search(x, k)
                    self.batches += 1
                    self.rows += x.shape[0]
                    r = 0
                    for p in ps:
                        n = p.vec.shape[0]
                        p.D, p.I = D[r:r + n], I[r:r + n]
                        r += n
                except BaseException as e:  # noqa: BLE001 - handed to every caller
                    for p in ps:
                        p.err = e
                for p in ps:
                    p.done.set()


class IndexService:
    """Serve one resident ``FAISS`` store (index in HBM) over TCP."""

    def __init__(self, store: FAISS, address=("127.0.0.1", 0), *, authkey: bytes,
                 max_batch: int = 4096, save_root: Optional[str] = None,
                 read_only: bool = False):
        self.store = store
        self._lock = _RWLock()
        self._authkey = authkey = _check_authkey(authkey)
        self._save_root = os.path.realpath(save_root) if save_root is not None else None
        self._read_only = bool(read_only)
        self._listener = Listener(address, backlog=128, authkey=authkey)
        self.address = self._listener.address
        self._coalescer = _Coalescer(self, max_batch)
        self._threads: List[threading.Thread] = []
        self._closed = threading.Event()
        self._accept = threading.Thread(target=self._accept_loop, name="vsearch-accept",
                                        daemon=True)

    # -- lifecycle --------------------------------------------------------------------
    def start(self) -> "IndexService":
        self._accept.start()
        return self

    def serve_forever(self) -> None:
        self.start()
        self._closed.wait()

    def close(self) -> None:
        if self._closed.is_set():
            return
        self._closed.set()
        try:
            # unblock accept() with a throwaway connection
            Client(self.address, authkey=self._authkey).close()
        except Exception:  # noqa: BLE001
            pass
        self._listener.close()
        self._coalescer.stop()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.close()

    @property
    def stats(self) -> dict:
        return {"search_batches": self._coalescer.batches, "search_rows": self._coalescer.rows}

    def _accept_loop(self):
        while not self._closed.is_set():
            try:
                conn = self._listener.accept()
            except Exception:  # noqa: BLE001 - bad auth or listener closed
                if self._closed.is_set():
                    return
                continue
            if self._closed.is_set():
                conn.close()
                return
            t = threading.Thread(target=self._serve_conn, args=(conn,), daemon=True)
            t.start()
            self._threads.append(t)

    def _serve_conn(self, conn):
        with conn:
            while True:
                try:
                    frame = conn.recv_bytes()
                except (EOFError, OSError):
                    return
                try:
                    header, payload = _unpack(frame)
                    out_h, out_p = self._dispatch(header, payload)
                    out_h["ok"] = True
                except BaseException as e:  # noqa: BLE001 - reported to the client
                    out_h, out_p = {"ok": False, "etype": type(e).__name__, "msg": str(e)}, b""
                try:
                    conn.send_bytes(_pack(out_h, out_p))
                except (EOFError, OSError):
                    return

    # -- requests ---------------------------------------------------------------------
    def _vectors(self, header: dict, payload: memoryview) -> np.ndarray:
        n, d = header["shape"]
        if d != self.store.index.d:
            raise AssertionError(f"query dim {d} != index dim {self.store.index.d}")
        return np.frombuffer(payload, dtype="<f4", count=n * d).reshape(n, d).copy()

    def _write(self, fn, *a, **kw):
        self._lock.acquire_write()
        try:
            return fn(*a, **kw)
        finally:
            self._lock.release_write()

    def _read(self, fn, *a, **kw):
        self._lock.acquire_read()
        try:
            return fn(*a, **kw)
        finally:
            self._lock.release_read()

    def _save_path(self, folder_path: str) -> str:
        """save_local's target, confined to the server's save_root."""
        if self._save_root is None:
            raise PermissionError("save_local is disabled: the server has no save_root")
        target = os.path.realpath(os.path.join(self._save_root, str(folder_path)))
        if os.path.commonpath([target, self._save_root]) != self._save_root:
            raise PermissionError(f"save_local: {folder_path!r} is outside the save root")
        return target

    def _dispatch(self, h: dict, payload: memoryview):
        op = h["op"]
        st = self.store
        if self._read_only and op in _WRITE_OPS:
            raise PermissionError(f"{op}: the service is read-only")
        if op == "info":
            return self._read(lambda: {"ntotal": st.index.ntotal, "d": st.index.d,
                                       "metric_type": st.index.metric_type,
                                       "distance_strategy": st.distance_strategy.value}), b""
        if op == "search":  # faiss-level: (n, d) -> D (n, k) f32, I (n, k) i64
            x = self._vectors(h, payload)
            D, I = self._read(self._coalescer.submit, x, int(h["k"]))
            return {"shape": list(D.shape)}, (np.ascontiguousarray(D, "<f4").tobytes()
                                              + np.ascontiguousarray(I, "<i8").tobytes())
        if op == "similarity_search_with_score":
            if "query" in h:
                vec = np.asarray([st._embed_query(h["query"])], dtype=np.float32)
            else:
                vec = self._vectors(h, payload)
            return {"results": self._search_docs(vec, h)}, b""
        if op == "embed_query":
            return {"vector": [float(v) for v in st._embed_query(h["query"])]}, b""
        if op == "add_texts":
            return {"ids": self._write(st.add_texts, h["texts"], metadatas=h.get("metadatas"),
                                       ids=h.get("ids"))}, b""
        if op == "upsert_texts":
            return {"ids": self._write(st.upsert_texts, h["texts"], h["metadatas"],
                                       key=h.get("key", "book_id"), ids=h.get("ids"))}, b""
        if op == "delete":
            return {"result": self._write(st.delete, h["ids"])}, b""
        if op == "get_by_ids":
            docs = self._read(st.get_by_ids, h["ids"])
            return {"docs": [d.to_json() for d in docs]}, b""
        if op == "save_local":
            name = str(h.get("index_name", "index"))
            if os.path.basename(name) != name or name in ("", ".", ".."):
                raise PermissionError(f"save_local: bad index_name {name!r}")
            self._write(st.save_local, self._save_path(h["folder_path"]), name)
            return {}, b""
        if op == "reconstruct":
            v = self._read(st.index.reconstruct, int(h["key"]))
            return {"shape": [int(v.shape[0])]}, np.ascontiguousarray(v, "<f4").tobytes()
        raise ValueError(f"unknown op {op!r}")

    def _search_docs(self, vec: np.ndarray, h: dict) -> List[list]:
        """FAISS.similarity_search_with_score_by_vector with the engine call coalesced
        (same filter / fetch_k / score_threshold semantics)."""
        st = self.store
        k = int(h.get("k", 4))
        flt = h.get("filter")
        if st._normalize_L2:
            from . import faiss as vfaiss
            vfaiss.normalize_L2(vec)
        filter_func = _create_filter_func(flt) if flt is not None else None
        docs = []
        self._lock.acquire_read()  # held from the search to the docstore lookup
        try:
            D, I = self._coalescer.submit(vec, k if flt is None else int(h.get("fetch_k", 20)))
            for s, i in zip(D[0], I[0]):
                if i == -1:
                    continue
                _id = st.index_to_docstore_id.get(int(i))
                doc = st.docstore.search(_id) if _id is not None else None
                if not isinstance(doc, Document):
                    raise ValueError(f"Could not find document for id {_id}, got {doc}")
                if filter_func is None or filter_func(doc.metadata):
                    docs.append((doc, float(s)))
        finally:
            self._lock.release_read()
        thr = h.get("score_threshold")
        if thr is not None:
            ip = st.distance_strategy.value in ("MAX_INNER_PRODUCT", "JACCARD")
            docs = [(d, s) for d, s in docs if (s >= thr if ip else s <= thr)]
        return [[d.to_json(), s] for d, s in docs[:k]]


class _RemoteIndex:
    """``store.index`` seen through the service: ntotal / d / metric_type / search."""

    def __init__(self, client: "RemoteFAISS"):
        self._c = client

    @property
    def ntotal(self) -> int:
        return int(self._c._call({"op": "info"})[0]["ntotal"])

    @property
    def d(self) -> int:
        return int(self._c._call({"op": "info"})[0]["d"])

    @property
    def metric_type(self) -> int:
        return int(self._c._call({"op": "info"})[0]["metric_type"])

    def search(self, x, k: int):
        x = np.ascontiguousarray(np.atleast_2d(np.asarray(x, dtype=np.float32)))
        h, p = self._c._call({"op": "search", "k": int(k), "shape": list(x.shape)},
                             x.astype("<f4").tobytes())
        n, kk = h["shape"]
        D = np.frombuffer(p, dtype="<f4", count=n * kk).reshape(n, kk).astype(np.float32)
        I = np.frombuffer(p[n * kk * 4:], dtype="<i8", count=n * kk).reshape(n, kk).astype(np.int64)
        return D, I

    def reconstruct(self, key: int) -> np.ndarray:
        h, p = self._c._call({"op": "reconstruct", "key": int(key)})
        return np.frombuffer(p, dtype="<f4", count=h["shape"][0]).astype(np.float32)


class RemoteFAISS:
    """Client with the LangChain ``FAISS`` surface the reference's call sites use
    (mcp_book_server.py:142, candidate_builder.py:321, book_vector/main.py:148, ...).
    Thread-safe (one request in flight per connection)."""

    def __init__(self, address, authkey: bytes):
        self._conn = Client(tuple(address) if isinstance(address, list) else address,
                            authkey=_check_authkey(authkey))
        self._mu = threading.Lock()
        self.index = _RemoteIndex(self)

    def close(self):
        self._conn.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _call(self, header: dict, payload: bytes = b""):
        with self._mu:
            self._conn.send_bytes(_pack(header, payload))
            h, p = _unpack(self._conn.recv_bytes())
        if not h.pop("ok"):
            raise _ERRORS.get(h["etype"], RuntimeError)(h["msg"])
        return h, p

    # -- reads ---------------------------------------------------------------------------
    @staticmethod
    def _results(h) -> List[Tuple[Document, np.float32]]:
        return [(Document.from_json(d), np.float32(s)) for d, s in h["results"]]

    def _search(self, header: dict, payload: bytes = b""):
        if callable(header.get("filter")):
            raise ValueError("RemoteFAISS: filter must be a dict (callables cannot travel)")
        return self._results(self._call(header, payload)[0])

    def similarity_search_with_score_by_vector(self, embedding, k: int = 4, filter=None,
                                               fetch_k: int = 20, **kwargs):
        v = np.ascontiguousarray(np.asarray([embedding], dtype=np.float32))
        return self._search({"op": "similarity_search_with_score", "k": k, "filter": filter,
                             "fetch_k": fetch_k, "score_threshold": kwargs.get("score_threshold"),
                             "shape": list(v.shape)}, v.astype("<f4").tobytes())

    def similarity_search_with_score(self, query: str, k: int = 4, filter=None,
                                     fetch_k: int = 20, **kwargs):
        return self._search({"op": "similarity_search_with_score", "query": query, "k": k,
                             "filter": filter, "fetch_k": fetch_k,
                             "score_threshold": kwargs.get("score_threshold")})

    def similarity_search_by_vector(self, embedding, k: int = 4, filter=None, fetch_k: int = 20,
                                    **kwargs) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score_by_vector(
            embedding, k, filter=filter, fetch_k=fetch_k, **kwargs)]

    def similarity_search(self, query: str, k: int = 4, filter=None, fetch_k: int = 20,
                          **kwargs) -> List[Document]:
        return [d for d, _ in self.similarity_search_with_score(
            query, k, filter=filter, fetch_k=fetch_k, **kwargs)]

    def get_by_ids(self, ids: Sequence[str]) -> List[Document]:
        return [Document.from_json(d) for d in self._call({"op": "get_by_ids",
                                                           "ids": list(ids)})[0]["docs"]]

    # -- writes --------------------------------------------------------------------------
    def add_texts(self, texts, metadatas: Optional[List[dict]] = None,
                  ids: Optional[List[str]] = None, **kwargs) -> List[str]:
        return self._call({"op": "add_texts", "texts": list(texts), "metadatas": metadatas,
                           "ids": ids})[0]["ids"]

    def upsert_texts(self, texts, metadatas: List[dict], key: str = "book_id",
                     ids: Optional[List[str]] = None, **kwargs) -> List[str]:
        return self._call({"op": "upsert_texts", "texts": list(texts), "metadatas": metadatas,
                           "key": key, "ids": ids})[0]["ids"]

    def delete(self, ids: Optional[List[str]] = None, **kwargs) -> Optional[bool]:
        if ids is None:
            raise ValueError("No ids provided to delete.")
        return self._call({"op": "delete", "ids": list(ids)})[0]["result"]

    def save_local(self, folder_path: str, index_name: str = "index") -> None:
        """Saved on the server, under its save_root (folder_path is relative to it)."""
        self._call({"op": "save_local", "folder_path": str(folder_path),
                    "index_name": index_name})


def serve(folder_path: str, embeddings, host: str = "127.0.0.1", port: int = 0, *,
          authkey: bytes, device: Optional[int] = None, max_batch: int = 4096,
          save_root: Optional[str] = None, read_only: bool = False) -> IndexService:
    """Load a saved store once (``FAISS.load_local``) and serve it until closed."""
    store = FAISS.load_local(folder_path, embeddings, allow_dangerous_deserialization=True,
                             device=device)
    return IndexService(store, (host, port), authkey=authkey, max_batch=max_batch,
                        save_root=save_root, read_only=read_only)


def main(argv=None):  # pragma: no cover - CLI wrapper
    from .synth import SynthEmbeddings

    ap = argparse.ArgumentParser(description="serve a saved vsearch store from HBM")
    ap.add_argument("folder")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8765)
    ap.add_argument("--device", type=int, default=None)
    ap.add_argument("--dim", type=int, default=1536)
    ap.add_argument("--save-root", default=None, help="directory save_local may write into")
    ap.add_argument("--read-only", action="store_true")
    a = ap.parse_args(argv)
    key = os.environ.get("VSEARCH_AUTHKEY", "")
    if not key:
        raise SystemExit("set VSEARCH_AUTHKEY to the shared secret (no default)")
    svc = serve(a.folder, SynthEmbeddings(a.dim), a.host, a.port, authkey=key.encode(),
                device=a.device, save_root=a.save_root, read_only=a.read_only)
    logger.warning("vsearch service on %s:%s", *svc.address)
    svc.serve_forever()


if __name__ == "__main__":  # pragma: no cover
    main()
