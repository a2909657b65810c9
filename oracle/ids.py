"""ORACLE — ctypes front of oracle/ids_oracle.c (C restatement of MCM.get_ids_shuffle,
reference models/Compression/MCM.py:364-423).  Test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
_SRC = os.path.join(_DIR, "ids_oracle.c")
_LIB = os.path.join(_DIR, "lib", "libids_oracle.so")
_handle = None


def build() -> str:
    """gcc the C restatement (no FP contraction: every fused op in it is an explicit fmaf)."""
    os.makedirs(os.path.dirname(_LIB), exist_ok=True)
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(_SRC):
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-shared", "-o", _LIB, _SRC, "-lm"], check=True)
    return _LIB


def _lib():
    global _handle
    if _handle is None:
        if not os.path.exists(_LIB):
            build()
        h = ctypes.CDLL(_LIB)
        h.oracle_ids_shuffle.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p]
        h.oracle_ids_shuffle.restype = ctypes.c_int
        h.oracle_torch_sum_f32.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        h.oracle_torch_sum_f32.restype = ctypes.c_float
        _handle = h
    return _handle


def ids_shuffle(scores: np.ndarray, K: int, lanes: int = 8):
    """scores [N, L] float32 -> (ids_shuffle, ids_restore) int64 [N, L]."""
    s = np.ascontiguousarray(scores, dtype=np.float32)
    if s.ndim == 1:
        s = s[None]
    n, L = s.shape
    shuf = np.empty((n, L), dtype=np.int64)
    rest = np.empty((n, L), dtype=np.int64)
    rc = _lib().oracle_ids_shuffle(s.ctypes.data, n, L, K, lanes, shuf.ctypes.data, rest.ctypes.data)
    if rc:
        raise ValueError("Number of patches should not be greater than the length of scores")
    return shuf, rest


def torch_sum_f32(x: np.ndarray, lanes: int = 8) -> float:
    x = np.ascontiguousarray(x, dtype=np.float32)
    return float(_lib().oracle_torch_sum_f32(x.ctypes.data, len(x), lanes))
