"""CPU: libvsearch.so loads and exports exactly the C-ABI that include/vsearch.h
declares; the ctypes signatures match the header.  No compute calls (no GPU here)."""

import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "vsearch.h")


def header_functions():
    text = open(HEADER, encoding="utf-8").read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?(?:int|char\s*\*|const\s+char\s*\*)\s*\**\s*(vs_\w+)\s*\(",
                       text, flags=re.M)
    return sorted(set(names))


def test_header_parses():
    names = header_functions()
    assert "vs_search" in names and "vs_last_error" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    from vsearch import _lib

    lib = _lib.load()
    for name in header_functions():
        assert hasattr(lib, name), name


def test_ctypes_table_matches_header():
    from vsearch import _lib

    assert sorted(_lib.SIGNATURES) == header_functions()


def test_header_arg_counts_match_ctypes():
    from vsearch import _lib

    text = open(HEADER, encoding="utf-8").read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    for name, (_, args) in _lib.SIGNATURES.items():
        m = re.search(name + r"\s*\(([^)]*)\)", text)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == len(args), (name, params, args)


def test_constants_match_header():
    from vsearch import _lib

    text = open(HEADER, encoding="utf-8").read()

    def const(name):
        return int(re.search(r"#define\s+" + name + r"\s+\(?(-?\d+)\)?", text).group(1))

    assert const("VS_METRIC_INNER_PRODUCT") == _lib.METRIC_INNER_PRODUCT == 0
    assert const("VS_METRIC_L2") == _lib.METRIC_L2 == 1
    assert const("VS_IN_DEVICE") == _lib.IN_DEVICE
    assert const("VS_OUT_DEVICE") == _lib.OUT_DEVICE
    assert const("VS_MAX_K") == _lib.MAX_K
    assert const("VS_E_INVALID") == _lib.E_INVALID


def test_error_path_without_device():
    """On a host with no GPU the library reports an error instead of falling back."""
    from vsearch import _lib

    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    lib = _lib.load()
    h = ctypes.c_void_p()
    rc = lib.vs_create(8, 1, 0, 0, ctypes.byref(h))
    assert rc != 0
    assert "device" in _lib.last_error()
    from vsearch import faiss as vfaiss

    with pytest.raises(RuntimeError):
        vfaiss.IndexFlatL2(8)


def test_argument_validation_is_host_side():
    from vsearch import _lib

    lib = _lib.load()
    assert lib.vs_create(0, 1, 0, 0, ctypes.byref(ctypes.c_void_p())) == _lib.E_INVALID
    assert lib.vs_create(8, 7, 0, 0, ctypes.byref(ctypes.c_void_p())) == _lib.E_INVALID
    assert lib.vs_search(None, None, 1, 1, None, None, 0, None) == _lib.E_INVALID
    assert lib.vs_merge_topk(None, None, 0, 1, 1, 1, 1, None, None, None) == _lib.E_INVALID
    assert "bad sizes" in _lib.last_error()
