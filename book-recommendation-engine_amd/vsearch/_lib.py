"""ctypes binding of libvsearch.so (C-ABI declared in include/vsearch.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
book-recommendation-engine_amd/csrc``).  There is deliberately no fallback: if
the library is missing or a call fails, the error surfaces as an exception, the
way faiss's SWIG layer raises ``RuntimeError`` from a ``FaissException``.
"""

from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("VSEARCH_LIB", os.path.join(_HERE, "libvsearch.so"))

METRIC_INNER_PRODUCT = 0
METRIC_L2 = 1
DTYPE_F32 = 0
DTYPE_BF16 = 1
IN_DEVICE = 1
OUT_DEVICE = 2
RAW_ORDER = 4
MAX_K = 64
ENGINE_AUTO = 0
ENGINE_FP32_MFMA = 1
ENGINE_BF16_VERIFY = 3
ENGINE_I8_VERIFY = 4

E_INVALID = -1
E_HIP = -2
E_OOM = -3
E_UNSUPPORTED = -4

_c_i64 = ctypes.c_int64
_c_int = ctypes.c_int
_vp = ctypes.c_void_p
_fp = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)

# name -> (restype, argtypes); kept in sync with include/vsearch.h (tests check both ways).
SIGNATURES = {
    "vs_last_error": (ctypes.c_char_p, []),
    "vs_version": (_c_int, []),
    "vs_device_count": (_c_int, [ctypes.POINTER(_c_int)]),
    "vs_create": (_c_int, [_c_int, _c_int, _c_int, _c_int, ctypes.POINTER(_vp)]),
    "vs_destroy": (_c_int, [_vp]),
    "vs_reserve": (_c_int, [_vp, _c_i64]),
    "vs_add": (_c_int, [_vp, _vp, _c_i64, _c_int, _vp]),
    "vs_add_synthetic": (_c_int, [_vp, _c_i64, ctypes.c_uint64, _c_i64, _vp]),
    "vs_add_synthetic_ids": (_c_int, [_vp, _vp, _c_i64, ctypes.c_uint64, _vp]),
    "vs_reset": (_c_int, [_vp]),
    "vs_ntotal": (_c_int, [_vp, _i64p]),
    "vs_dim": (_c_int, [_vp, ctypes.POINTER(_c_int)]),
    "vs_metric": (_c_int, [_vp, ctypes.POINTER(_c_int)]),
    "vs_dtype": (_c_int, [_vp, ctypes.POINTER(_c_int)]),
    "vs_set_id_base": (_c_int, [_vp, _c_i64]),
    "vs_set_engine": (_c_int, [_vp, _c_int]),
    "vs_filter_plane": (_c_int, [_vp, ctypes.POINTER(_c_int)]),
    "vs_notice": (ctypes.c_char_p, [_vp]),
    "vs_search": (_c_int, [_vp, _vp, _c_i64, _c_i64, _vp, _vp, _c_int, _vp]),
    "vs_reconstruct_n": (_c_int, [_vp, _c_i64, _c_i64, _vp, _c_int, _vp]),
    "vs_remove_ids": (_c_int, [_vp, _vp, _c_i64, _i64p]),
    "vs_selfjoin": (
        _c_int,
        [_vp, _c_i64, _c_i64, _c_i64, _c_int, ctypes.c_float, _vp, _vp, _c_int, _vp],
    ),
    "vs_merge_topk": (
        _c_int,
        [_vp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_int, _vp, _vp, _vp],
    ),
    "vs_fill_synthetic": (_c_int, [_vp, _c_i64, _c_i64, ctypes.c_uint64, _c_i64, _vp]),
    "vs_timer_enable": (_c_int, [_c_int]),
    "vs_timer_reset": (_c_int, []),
    "vs_timer_read": (_c_int, [ctypes.POINTER(ctypes.c_double), _i64p]),
    "vs_timer_kernel": (ctypes.c_char_p, []),
    "vs_timer_read_kernel": (_c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), _i64p]),
    "vs_timer_read_kernel_share": (_c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                            _i64p, ctypes.POINTER(ctypes.c_double)]),
    "vs_x1_stamps": (_c_int, [ctypes.POINTER(ctypes.c_ulonglong), _c_int]),
    "vs_filter_stats": (_c_int, [_i64p, _i64p, _c_int]),
    "vs_filter_wide_stats": (_c_int, [_i64p]),
    "vs_filter_second_stats": (_c_int, [_i64p]),
    "vs_filter_exact_stats": (_c_int, [_i64p]),
    "vs_filter_wide_sets": (_c_int, [_i64p, _i64p]),
    "vs_filter_dump_stats": (_c_int, [_i64p, _i64p]),
}

_lock = threading.Lock()
_lib = None


def _preload_hip_runtime() -> None:
    """Use ONE HIP runtime per process.  PyTorch-ROCm ships its own
    libamdhip64.so (soname libamdhip64.so.7) and loads it by path; if
    libvsearch.so pulled /opt/rocm's copy in first, the process would hold two
    HIP/HSA runtimes and torch's would fail to initialise.  When torch is
    installed, its runtime is loaded first (RTLD_GLOBAL) so libvsearch binds to
    it by soname; torch itself is not imported."""
    if os.environ.get("VSEARCH_SYSTEM_HIP"):
        return
    try:
        import importlib.util

        spec = importlib.util.find_spec("torch")
    except Exception:
        return
    if spec is None or not spec.submodule_search_locations:
        return
    path = os.path.join(list(spec.submodule_search_locations)[0], "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


class VSearchError(RuntimeError):
    """A libvsearch call failed (faiss raises RuntimeError in the same places)."""

    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code


def load():
    """Load libvsearch.so once; raise loudly if it is not built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libvsearch.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
            )
        _preload_hip_runtime()
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    msg = load().vs_last_error()
    return msg.decode("utf-8", "replace") if msg else ""


def check(rc: int, what: str = "") -> None:
    """Turn a VS_E* status into the exception faiss/numpy callers expect."""
    if rc == 0:
        return
    msg = last_error() or what
    if rc == E_INVALID:
        # faiss: FAISS_THROW_IF_NOT -> RuntimeError (python asserts are raised
        # by the wrappers before reaching here).
        raise VSearchError(rc, msg)
    raise VSearchError(rc, msg)


def device_count() -> int:
    n = _c_int(0)
    rc = load().vs_device_count(ctypes.byref(n))
    if rc != 0:
        return 0
    return n.value


def timer_enable(on: bool = True) -> None:
    check(load().vs_timer_enable(1 if on else 0))


def timer_reset() -> None:
    check(load().vs_timer_reset())


def timer_kernel() -> str:
    """Name of the fused search kernel launched by the last search."""
    return load().vs_timer_kernel().decode()


def timer_read():
    """(total_ms, launches) of the dominant search kernel since the last reset."""
    ms = ctypes.c_double(0.0)
    n = _c_i64(0)
    check(load().vs_timer_read(ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


def timer_read_kernel(name: str):
    """(summed kernel ms, launches) of the timed spans named `name`."""
    ms = ctypes.c_double(0.0)
    n = ctypes.c_int64(0)
    check(load().vs_timer_read_kernel(name.encode(), ctypes.byref(ms), ctypes.byref(n)))
    return ms.value, n.value


def timer_read_kernel_share(name: str):
    """(summed kernel ms, launches, summed share of their passes' tiles) of the
    timed spans named `name`."""
    ms = ctypes.c_double(0.0)
    n = ctypes.c_int64(0)
    sh = ctypes.c_double(0.0)
    check(load().vs_timer_read_kernel_share(name.encode(), ctypes.byref(ms), ctypes.byref(n),
                                            ctypes.byref(sh)))
    return ms.value, n.value, sh.value


def filter_stats(reset: bool = False):
    """(queries searched by the filter-and-verify engine, queries the exact
    engine redid) since the last reset."""
    q = ctypes.c_int64(0)
    f = ctypes.c_int64(0)
    check(load().vs_filter_stats(ctypes.byref(q), ctypes.byref(f), 1 if reset else 0))
    return q.value, f.value


def filter_wide_stats() -> int:
    """Flagged queries re-checked by the wide verification since the last
    filter_stats reset (read it before that reset)."""
    w = ctypes.c_int64(0)
    check(load().vs_filter_wide_stats(ctypes.byref(w)))
    return w.value


def filter_wide_sets():
    """(entries, rescored): wide-set entries summed over the wide-checked
    queries, and how many of them were read again and rescored, since the last
    filter_stats reset (read them before that reset)."""
    e = ctypes.c_int64(0)
    r = ctypes.c_int64(0)
    check(load().vs_filter_wide_sets(ctypes.byref(e), ctypes.byref(r)))
    return e.value, r.value


def filter_second_stats() -> int:
    """Queries handed from the int8 plane to the bf16 plane by the staged
    filter engine since the last filter_stats reset (read it before that reset)."""
    v = ctypes.c_int64(0)
    check(load().vs_filter_second_stats(ctypes.byref(v)))
    return v.value


def filter_exact_stats() -> int:
    """Queries the staged engine's last stage ranked over every row by the
    exact key (the fp32 bound could not prove its candidates) since the last
    filter_stats reset (read it before that reset)."""
    v = ctypes.c_int64(0)
    check(load().vs_filter_exact_stats(ctypes.byref(v)))
    return v.value


def filter_dump_stats():
    """(dumps, overflows): blocks the filter pass's dump launches stored and
    lane lists that ran out of dump slots (their queries went to the next
    stage) since the last filter_stats reset (read them before that reset)."""
    d = ctypes.c_int64(0)
    o = ctypes.c_int64(0)
    check(load().vs_filter_dump_stats(ctypes.byref(d), ctypes.byref(o)))
    return d.value, o.value
