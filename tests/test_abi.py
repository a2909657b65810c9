"""The C-ABI library: loads without a GPU, exports every symbol include/tmae.h declares, and
validates arguments on the host (errors surface as the reference's exceptions).  CPU only."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "tmae.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(tmae_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "tmae_ids_shuffle" in names and "tmae_mha_fwd" in names and len(names) >= 18


def test_library_exports_every_declared_symbol(tmae):
    lib = tmae.load_library()
    from textmae_amd import _lib

    for name in declared_functions():
        assert hasattr(lib, name), name
        if name != "tmae_last_error_string":
            assert name in _lib.SIGNATURES or name in _lib.VALUE_FUNCS, f"{name} has no ctypes signature"


def test_abi_version(tmae):
    lib = tmae.load_library()
    assert lib.tmae_abi_version() == 1


def test_host_side_validation(tmae):
    """shape checks run before any device work, so they are testable without a GPU"""
    from textmae_amd import _lib

    with pytest.raises(ValueError, match="Number of patches should not be greater"):
        _lib.call("tmae_ids_shuffle", None, None, None, 2, 16, 17, 8, None)
    with pytest.raises(ValueError, match="head dim"):
        _lib.call("tmae_mha_fwd", None, None, 1, 10, 2, 48, ctypes.c_float(1.0), 0, None)
    a = _lib.ConvArgs()
    a.c1, a.ld1, a.n, a.H, a.W, a.stride, a.cout, a.nb1, a.nb2, a.y_f32 = 20, 20, 1, 4, 4, 1, 8, 1, 1, 1
    with pytest.raises(ValueError, match="multiples of"):
        _lib.call("tmae_conv3x3", ctypes.byref(a), 1, None)
    with pytest.raises(ValueError, match="K=30"):
        _lib.call("tmae_linear_fwd", None, 0, 30, 1, 0, 0, None, None, None, 0, 8, None, 0, 4, 8, 30, 0, 1, None)


def test_missing_library_fails_loudly(tmae, monkeypatch):
    from textmae_amd import _lib

    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", "/nonexistent/libtmae.so")
    with pytest.raises(_lib.TmaeError):
        _lib.load()
