"""faiss-compatible flat indexes backed by the MI355X engine (libvsearch.so).

Drop-in for the subset of faiss-cpu 1.11.0 (/root/reference/poetry.lock:866-867,
not vendored) that the reference reaches through LangChain's ``FAISS`` store:

* ``IndexFlatL2(d)`` / ``IndexFlatIP(d)`` — built by ``FAISS.from_texts``
  (src/ingestion_service/pipeline.py:359, src/incremental_workers/book_vector/main.py:121,469)
* ``index.add`` (via ``FAISS.add_texts``, pipeline.py:363, book_vector/main.py:148)
* ``index.search`` (the only search call, inside
  ``similarity_search_with_score_by_vector``; reached from
  src/recommendation_api/mcp_book_server.py:142, candidate_builder.py:187,321, service.py:529,627)
* ``index.ntotal`` (pipeline.py:186,524; book_vector/main.py:162-170,349-410)
* ``index.reconstruct(i)`` (candidate_builder.py:166-168, service.py:490-494)
* ``index.remove_ids`` (via ``FAISS.delete``)
* ``write_index`` / ``read_index`` (via ``save_local`` / ``load_local``)
* ``normalize_L2`` (LangChain's ``normalize_L2=True`` option)

Argument checks mirror faiss's python wrapper (``assert d == self.d``,
``assert k > 0``); library failures raise ``RuntimeError`` subclasses.
The rows live in HBM of one device; there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

from . import _lib
from ._lib import METRIC_INNER_PRODUCT, METRIC_L2, VSearchError

__all__ = [
    "METRIC_INNER_PRODUCT",
    "METRIC_L2",
    "Index",
    "IndexFlat",
    "IndexFlatIP",
    "IndexFlatL2",
    "IDSelectorBatch",
    "normalize_L2",
    "read_index",
    "write_index",
    "default_device",
]


def default_device() -> int:
    """Device used by indexes created without an explicit ``device``: $VS_DEVICE,
    else $LOCAL_RANK (one process per GPU), else 0."""
    for var in ("VS_DEVICE", "LOCAL_RANK"):
        v = os.environ.get(var)
        if v is not None and v.strip() != "":
            return int(v)
    return 0


def _as_f32_rows(x, d=None):
    x = np.ascontiguousarray(x, dtype="float32")
    if x.ndim != 2:
        raise ValueError(f"expected a 2-D array, got shape {x.shape}")
    if d is not None:
        assert x.shape[1] == d
    return x


class IDSelectorBatch:
    """faiss.IDSelectorBatch: a set of labels (duplicates collapse)."""

    def __init__(self, ids):
        self.ids = np.unique(np.ascontiguousarray(ids, dtype="int64").ravel())

    def is_member(self, i: int) -> bool:
        return bool(np.isin(i, self.ids))


class Index:
    """Common base (faiss.Index)."""

    is_trained = True


class IndexFlat(Index):
    """Exact flat index (faiss::IndexFlat) on one GPU.

    ``dtype="bf16"`` stores rows as bf16 (round to nearest even) — half the HBM
    of fp32, for corpora that do not fit otherwise (BASELINE config 5).  Queries
    are rounded to bf16 as well and products accumulate in fp32, so the search is
    exact over the rounded vectors; against fp32 vectors it is reported as
    recall@k.  ``reconstruct`` returns the stored (rounded) values.
    """

    def __init__(self, d: int, metric: int = METRIC_L2, *, device: int | None = None,
                 dtype: str = "f32"):
        d = int(d)
        self._lib = _lib.load()
        self._h = ctypes.c_void_p()
        self._device = default_device() if device is None else int(device)
        code = {"f32": _lib.DTYPE_F32, "float32": _lib.DTYPE_F32,
                "bf16": _lib.DTYPE_BF16, "bfloat16": _lib.DTYPE_BF16}[dtype]
        _lib.check(self._lib.vs_create(d, int(metric), code, self._device, ctypes.byref(self._h)),
                   "vs_create")
        self._d = d
        self._metric = int(metric)
        self._dtype = "bf16" if code == _lib.DTYPE_BF16 else "f32"

    # -- attributes faiss exposes -------------------------------------------------
    @property
    def d(self) -> int:
        return self._d

    @property
    def metric_type(self) -> int:
        return self._metric

    @property
    def device(self) -> int:
        return self._device

    @property
    def dtype(self) -> str:
        return self._dtype

    @property
    def ntotal(self) -> int:
        n = ctypes.c_int64(0)
        _lib.check(self._lib.vs_ntotal(self._h, ctypes.byref(n)), "vs_ntotal")
        return n.value

    def __len__(self) -> int:  # convenience; faiss has no __len__
        return self.ntotal

    def __del__(self):
        # no module-global lookups here: at interpreter exit `ctypes` may already
        # be torn down; the handle object itself is cleared in place
        h = getattr(self, "_h", None)
        if h is None or not h.value:
            return
        try:
            self._lib.vs_destroy(h)
        except Exception:  # interpreter shutdown: the library may be gone
            pass
        h.value = None

    # -- mutation ---------------------------------------------------------------------
    def add(self, x) -> None:
        """faiss Index.add: append rows (labels ntotal, ntotal+1, ...)."""
        x = _as_f32_rows(x, self._d)
        n = x.shape[0]
        if n == 0:
            return
        _lib.check(self._lib.vs_add(self._h, x.ctypes.data, n, 0, None), "vs_add")

    def add_device(self, ptr: int, n: int, stream: int = 0) -> None:
        """Append n rows already in device memory (row-major float32, stride d)."""
        _lib.check(self._lib.vs_add(self._h, ctypes.c_void_p(ptr), int(n), _lib.IN_DEVICE,
                                    ctypes.c_void_p(stream)), "vs_add")

    def add_synthetic(self, n: int, seed: int, row0: int = 0, stream: int = 0) -> None:
        """Append the counter-based synthetic rows row0..row0+n-1 (see vsearch.synth)."""
        _lib.check(self._lib.vs_add_synthetic(self._h, int(n), ctypes.c_uint64(seed),
                                              int(row0), ctypes.c_void_p(stream)),
                   "vs_add_synthetic")

    def add_synthetic_ids(self, ids, seed: int, stream: int = 0) -> None:
        """Append the synthetic corpus rows with generator row numbers `ids`."""
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        if ids.size:
            _lib.check(self._lib.vs_add_synthetic_ids(self._h, ids.ctypes.data, ids.size,
                                                      ctypes.c_uint64(seed),
                                                      ctypes.c_void_p(stream)),
                       "vs_add_synthetic_ids")

    def reserve(self, n: int) -> None:
        _lib.check(self._lib.vs_reserve(self._h, int(n)), "vs_reserve")

    def reset(self) -> None:
        _lib.check(self._lib.vs_reset(self._h), "vs_reset")

    def remove_ids(self, x) -> int:
        """faiss IndexFlat.remove_ids: stable compaction; returns #removed."""
        if isinstance(x, IDSelectorBatch):
            ids = x.ids
        else:
            ids = np.ascontiguousarray(x, dtype="int64")
            assert ids.ndim == 1
        nrem = ctypes.c_int64(0)
        if ids.size == 0:
            return 0
        _lib.check(self._lib.vs_remove_ids(self._h, ids.ctypes.data, ids.size,
                                           ctypes.byref(nrem)), "vs_remove_ids")
        return int(nrem.value)

    def set_engine(self, engine: str) -> None:
        """Large-batch arithmetic of fp32 indexes: "auto" (filter and verify in
        stages: the int8 plane, then the bf16 plane for what int8 cannot settle,
        then the exact fp32 engine), "fp32" (the exact fp32 MFMA engine), "i8v"
        or "bf16v" (filter and verify on that plane alone, then fp32)."""
        code = {"auto": _lib.ENGINE_AUTO, "fp32": _lib.ENGINE_FP32_MFMA,
                "bf16v": _lib.ENGINE_BF16_VERIFY, "i8v": _lib.ENGINE_I8_VERIFY}[engine]
        _lib.check(self._lib.vs_set_engine(self._h, code), "vs_set_engine")

    @property
    def filter_planes(self):
        """The filter planes of this index, in the order the staged engine runs
        them: ("i8", "bf16") for inner-product and L2 fp32 indexes (L2 as an
        augmented inner product), ("bf16",) for cosine, () for bf16 indexes
        (which search their stored values exactly)."""
        v = ctypes.c_int(0)
        _lib.check(self._lib.vs_filter_plane(self._h, ctypes.byref(v)), "vs_filter_plane")
        return tuple(n for bit, n in ((1, "i8"), (2, "bf16")) if v.value & bit)

    @property
    def notice(self) -> str:
        """The library's last notice for this index ("" if none): a filter plane
        dropped because HBM ran short while the storage grew."""
        v = self._lib.vs_notice(self._h)
        return v.decode() if v else ""

    def set_id_base(self, base: int) -> None:
        _lib.check(self._lib.vs_set_id_base(self._h, int(base)), "vs_set_id_base")

    # -- queries -----------------------------------------------------------------------
    def search(self, x, k, *, D=None, I=None, raw: bool = False):
        """faiss Index.search: returns (D float32 (n,k), I int64 (n,k)).

        ``raw=True`` returns the k lexicographically best (key, label) entries
        instead of faiss's inner-product tie order (VS_RAW_ORDER; the per-shard
        half of an exact sharded search, see vsearch.sharded)."""
        x = _as_f32_rows(x)
        n, d = x.shape
        assert d == self._d
        k = int(k)
        assert k > 0
        if D is None:
            D = np.empty((n, k), dtype=np.float32)
        else:
            assert D.shape == (n, k)
        if I is None:
            I = np.empty((n, k), dtype=np.int64)
        else:
            assert I.shape == (n, k)
        if n == 0:
            return D, I
        _lib.check(self._lib.vs_search(self._h, x.ctypes.data, n, k, D.ctypes.data,
                                       I.ctypes.data, _lib.RAW_ORDER if raw else 0, None),
                   "vs_search")
        return D, I

    def search_device(self, xq_ptr: int, n: int, k: int, D_ptr: int, I_ptr: int,
                      stream: int = 0, raw: bool = False) -> None:
        """Device-resident search: all buffers are device pointers on this index's
        device; stream-ordered on `stream` (a hipStream_t, 0 = default stream).
        Returns once the first filter stage's count of unsettled queries is read
        (later stages are enqueued only for queries left; VS_TAIL_WAIT=0 keeps
        the call fully asynchronous)."""
        flags = _lib.IN_DEVICE | _lib.OUT_DEVICE | (_lib.RAW_ORDER if raw else 0)
        _lib.check(self._lib.vs_search(self._h, ctypes.c_void_p(xq_ptr), int(n), int(k),
                                       ctypes.c_void_p(D_ptr), ctypes.c_void_p(I_ptr), flags,
                                       ctypes.c_void_p(stream)), "vs_search")

    def reconstruct(self, key) -> np.ndarray:
        """faiss Index.reconstruct(key) -> float32 (d,)."""
        key = int(key)
        out = np.empty((1, self._d), dtype=np.float32)
        _lib.check(self._lib.vs_reconstruct_n(self._h, key, 1, out.ctypes.data, 0, None),
                   "vs_reconstruct_n")
        return out[0]

    def reconstruct_n(self, n0: int = 0, ni: int = -1) -> np.ndarray:
        """faiss Index.reconstruct_n(n0, ni) -> float32 (ni, d)."""
        if ni == -1:
            ni = self.ntotal - int(n0)
        out = np.empty((int(ni), self._d), dtype=np.float32)
        if ni:
            _lib.check(self._lib.vs_reconstruct_n(self._h, int(n0), int(ni), out.ctypes.data, 0,
                                                  None), "vs_reconstruct_n")
        return out

    def selfjoin(self, k: int, *, q0: int = 0, nq: int | None = None,
                 exclude_self: bool = True, min_sim: float = -np.inf):
        """Cosine self-join over stored rows [q0, q0+nq) (pgvector `<=>` semantics):
        returns (S float32 (nq,k) similarities, I int64 (nq,k) labels, -1 = none)."""
        ntotal = self.ntotal
        nq = ntotal - q0 if nq is None else int(nq)
        k = int(k)
        assert k > 0
        S = np.empty((nq, k), dtype=np.float32)
        I = np.empty((nq, k), dtype=np.int64)
        if nq == 0:
            return S, I
        _lib.check(self._lib.vs_selfjoin(self._h, int(q0), nq, k, 1 if exclude_self else 0,
                                         ctypes.c_float(min_sim), S.ctypes.data, I.ctypes.data,
                                         0, None), "vs_selfjoin")
        return S, I

    def selfjoin_device(self, k: int, q0: int, nq: int, D_ptr: int, I_ptr: int, *,
                        exclude_self: bool = True, min_sim: float = -np.inf,
                        stream: int = 0) -> None:
        _lib.check(self._lib.vs_selfjoin(self._h, int(q0), int(nq), int(k),
                                         1 if exclude_self else 0, ctypes.c_float(min_sim),
                                         ctypes.c_void_p(D_ptr), ctypes.c_void_p(I_ptr),
                                         _lib.OUT_DEVICE, ctypes.c_void_p(stream)),
                   "vs_selfjoin")


class IndexFlatL2(IndexFlat):
    def __init__(self, d: int, **kw):
        super().__init__(d, METRIC_L2, **kw)


class IndexFlatIP(IndexFlat):
    def __init__(self, d: int, **kw):
        super().__init__(d, METRIC_INNER_PRODUCT, **kw)


def normalize_L2(x: np.ndarray) -> None:
    """faiss.normalize_L2 (fvec_renorm_L2): in place, rows with zero norm untouched."""
    if not (isinstance(x, np.ndarray) and x.dtype == np.float32 and x.flags.c_contiguous):
        raise TypeError("normalize_L2 expects a C-contiguous float32 numpy array")
    nr = np.einsum("ij,ij->i", x, x, dtype=np.float32)
    inv = np.ones_like(nr)
    pos = nr > 0
    inv[pos] = (1.0 / np.sqrt(nr[pos].astype(np.float32))).astype(np.float32)
    x *= inv[:, None]


# ---- persistence: faiss flat binary format ------------------------------------------
# faiss index_write.cpp for IndexFlat [upstream]: fourcc ("IxF2" L2 / "IxFI" IP), then
# write_index_header: d:int32, ntotal:int64, dummy:int64 (1<<20) x2, is_trained:uint8,
# metric_type:int32 (metric_arg:float32 only when metric_type > 1), then the codes
# vector as size:uint64 (= #floats) followed by the raw float32 rows.
_FOURCC = {METRIC_L2: b"IxF2", METRIC_INNER_PRODUCT: b"IxFI"}


def write_index(index: IndexFlat, fname) -> None:
    """faiss.write_index for flat indexes (streams rows out in bounded chunks)."""
    if not all(hasattr(index, a) for a in ("d", "ntotal", "metric_type", "reconstruct_n")) \
            or index.metric_type not in _FOURCC:
        raise TypeError("write_index: only flat L2 / inner-product indexes are supported")
    ntotal = index.ntotal
    with open(fname, "wb") as f:
        f.write(_FOURCC[index.metric_type])
        f.write(struct.pack("<iqqq?i", index.d, ntotal, 1 << 20, 1 << 20, True,
                            index.metric_type))
        f.write(struct.pack("<Q", ntotal * index.d))
        step = max(1, (64 << 20) // (4 * index.d))
        for i0 in range(0, ntotal, step):
            f.write(index.reconstruct_n(i0, min(step, ntotal - i0)).tobytes())


def read_index(fname, *, device: int | None = None, index_factory=None) -> IndexFlat:
    """faiss.read_index for flat indexes (IxF2 / IxFI / IxFl with metric 0|1).
    `index_factory(d, metric)` overrides the GPU index constructor (tests)."""
    with open(fname, "rb") as f:
        h = f.read(4)
        if h not in (b"IxF2", b"IxFI", b"IxFl"):
            raise RuntimeError(f"read_index: unsupported index type {h!r} (flat indexes only)")
        d, ntotal, _, _, _, metric = struct.unpack("<iqqq?i", f.read(4 + 8 * 3 + 1 + 4))
        if metric > 1:
            f.read(4)  # metric_arg
            raise RuntimeError(f"read_index: metric {metric} not supported")
        (size,) = struct.unpack("<Q", f.read(8))
        if size != ntotal * d:
            raise RuntimeError("read_index: codes size does not match d*ntotal")
        if index_factory is not None:
            index = index_factory(d, metric)
        else:
            index = IndexFlat(d, metric, device=device)
            if ntotal:
                index.reserve(ntotal)
        step = max(1, (64 << 20) // (4 * d))
        left = ntotal
        while left > 0:
            m = min(step, left)
            buf = f.read(4 * d * m)
            if len(buf) != 4 * d * m:
                raise RuntimeError("read_index: truncated file")
            index.add(np.frombuffer(buf, dtype="<f4").reshape(m, d))
            left -= m
    return index
