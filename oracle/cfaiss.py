"""ORACLE — ctypes binding of oracle/faiss_flat.c (faiss heap restatement).
Test infrastructure only; see oracle/flat.py for the rules."""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle_faiss.so")
_SO_SIMD = os.path.join(_HERE, "build", "liboracle_faiss_simd.so")
_lib = None
_lib_simd = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        lib = ctypes.CDLL(_SO)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.oracle_knn_seq.argtypes = [vp, vp, i64, i64, i64, i64, ctypes.c_int, vp, vp, vp]
        lib.oracle_knn_seq.restype = None
        lib.oracle_heap_select.argtypes = [vp, i64, i64, i64, ctypes.c_int, vp, vp]
        lib.oracle_heap_select.restype = None
        _lib = lib
    return _lib


def knn_seq(xb, xq, k: int, metric: int, valid=None):
    """faiss sequential branch (fp32 scalar sums, heap, heap_reorder)."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    vptr = None
    if valid is not None:
        valid = np.ascontiguousarray(valid, dtype=np.uint8)
        vptr = valid.ctypes.data
    load().oracle_knn_seq(xq.ctypes.data, xb.ctypes.data, d, nq, xb.shape[0], k, metric, vptr,
                          D.ctypes.data, I.ctypes.data)
    return D, I


def heap_select(scores, k: int, metric: int):
    """faiss heap discipline applied to given float32 scores (nq, ny)."""
    s = np.ascontiguousarray(scores, dtype=np.float32)
    nq, ny = s.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    load().oracle_heap_select(s.ctypes.data, nq, ny, k, metric, D.ctypes.data, I.ctypes.data)
    return D, I


def load_simd():
    global _lib_simd
    if _lib_simd is None:
        if not os.path.exists(_SO_SIMD):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        lib = ctypes.CDLL(_SO_SIMD)
        vp, i64 = ctypes.c_void_p, ctypes.c_int64
        lib.oracle_knn_seq_simd.argtypes = [vp, vp, i64, i64, i64, i64, ctypes.c_int, vp, vp]
        lib.oracle_knn_seq_simd.restype = None
        _lib_simd = lib
    return _lib_simd


def knn_seq_simd(xb, xq, k: int, metric: int):
    """faiss-SPEED stand-in for the nq = 1 baseline (oracle/faiss_flat_simd.c:
    reassociated 16-lane fp32 sums as faiss's FAISS_PRAGMA_IMPRECISE_LOOP
    builds, one thread).  Not a parity oracle: its scores round differently."""
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    xq = np.ascontiguousarray(xq, dtype=np.float32)
    nq, d = xq.shape
    D = np.empty((nq, k), dtype=np.float32)
    I = np.empty((nq, k), dtype=np.int64)
    load_simd().oracle_knn_seq_simd(xq.ctypes.data, xb.ctypes.data, d, nq, xb.shape[0], k,
                                    metric, D.ctypes.data, I.ctypes.data)
    return D, I
