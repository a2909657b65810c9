"""compressai's entropy-coder classes (``compressai.ans``) over the C ABI (csrc/rans.cpp).

Same names and call signatures as the objects the reference uses: ``BufferedRansEncoder``
(MCM.py:845, 882-887, 890), ``RansDecoder`` (MCM.py:917-918, 941-943), ``RansEncoder`` (used by
EntropyModel.compress) and ``pmf_to_quantized_cdf`` (EntropyModel._pmf_to_cdf).  Arguments may be
Python lists (the reference passes ``.tolist()`` results), numpy arrays or CPU tensors; symbol
arrays are handed to the coder without per-element Python work.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

__all__ = ["BufferedRansEncoder", "RansEncoder", "RansDecoder", "pmf_to_quantized_cdf"]


def _i32(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.int32))


def _tables(cdfs, cdf_sizes, offsets):
    if isinstance(cdfs, (list, tuple)) and cdfs and isinstance(cdfs[0], (list, tuple)):
        width = max(len(r) for r in cdfs)
        t = np.zeros((len(cdfs), width), dtype=np.int32)
        for i, r in enumerate(cdfs):
            t[i, :len(r)] = r
    else:
        t = _i32(cdfs)
    if t.ndim != 2:
        raise ValueError("cdfs must be a 2-D table [num_cdfs][cdf_length]")
    sizes, offs = _i32(cdf_sizes).reshape(-1), _i32(offsets).reshape(-1)
    if sizes.size != t.shape[0] or offs.size != t.shape[0]:
        raise ValueError(f"{t.shape[0]} cdfs but {sizes.size} sizes and {offs.size} offsets")
    return t, sizes, offs


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def pmf_to_quantized_cdf(pmf, precision: int = 16):
    p = np.ascontiguousarray(np.asarray(pmf.detach().cpu() if isinstance(pmf, torch.Tensor) else pmf,
                                        dtype=np.float32).reshape(-1))
    out = np.empty(p.size + 1, dtype=np.int32)
    _lib.call("tmae_pmf_to_quantized_cdf", _ptr(p), p.size, int(precision), _ptr(out))
    return out.tolist()


class BufferedRansEncoder:
    def __init__(self):
        h = ctypes.c_void_p()
        _lib.call("tmae_rans_encoder_create", ctypes.byref(h))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value and _lib._lib is not None:
            _lib._lib.tmae_rans_encoder_destroy(h)
            self._h = None

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_sizes, offsets):
        sym, idx = _i32(symbols).reshape(-1), _i32(indexes).reshape(-1)
        if sym.size != idx.size:
            raise ValueError(f"{sym.size} symbols but {idx.size} indexes")
        t, sizes, offs = _tables(cdfs, cdf_sizes, offsets)
        _lib.call("tmae_rans_encode_with_indexes", self._h, _ptr(sym), _ptr(idx), sym.size, _ptr(t), t.shape[1],
                  _ptr(sizes), _ptr(offs), t.shape[0])

    def flush(self) -> bytes:
        n = ctypes.c_longlong()
        _lib.call("tmae_rans_encoder_flush", self._h, ctypes.byref(n))
        buf = (ctypes.c_uint8 * n.value)()
        _lib.call("tmae_rans_encoder_take", self._h, buf, n.value)
        return bytes(buf)


class RansEncoder:
    """one-shot encoder (compressai RansEncoder.encode_with_indexes -> bytes)"""

    def encode_with_indexes(self, symbols, indexes, cdfs, cdf_sizes, offsets) -> bytes:
        enc = BufferedRansEncoder()
        enc.encode_with_indexes(symbols, indexes, cdfs, cdf_sizes, offsets)
        return enc.flush()


class RansDecoder:
    def __init__(self):
        self._h = None

    def _close(self):
        if self._h is not None and self._h.value and _lib._lib is not None:
            _lib._lib.tmae_rans_decoder_destroy(self._h)
        self._h = None

    def __del__(self):
        self._close()

    def set_stream(self, stream: bytes):
        self._close()
        data = bytes(stream)
        h = ctypes.c_void_p()
        _lib.call("tmae_rans_decoder_create", data, len(data), ctypes.byref(h))
        self._h = h

    def decode_stream_array(self, indexes, cdfs, cdf_sizes, offsets) -> np.ndarray:
        if self._h is None:
            raise ValueError("RansDecoder: set_stream() first")
        idx = _i32(indexes).reshape(-1)
        t, sizes, offs = _tables(cdfs, cdf_sizes, offsets)
        out = np.empty(idx.size, dtype=np.int32)
        _lib.call("tmae_rans_decode_with_indexes", self._h, _ptr(idx), idx.size, _ptr(t), t.shape[1], _ptr(sizes),
                  _ptr(offs), t.shape[0], _ptr(out))
        return out

    def decode_stream(self, indexes, cdfs, cdf_sizes, offsets):
        return self.decode_stream_array(indexes, cdfs, cdf_sizes, offsets).tolist()

    def decode_with_indexes(self, stream, indexes, cdfs, cdf_sizes, offsets):
        self.set_stream(stream)
        try:
            return self.decode_stream(indexes, cdfs, cdf_sizes, offsets)
        finally:
            self._close()
