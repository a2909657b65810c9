"""HuffmanCoding — drop-in for reference utils/huffman.py:6-171 (side information of the Kodak eval,
testing.py:71-74, 88-89): the same class surface (``compress(tensor) -> (bits, shape, device)``,
``decompress(bits, shape, device)``, ``encode`` / ``decode``, the ``codes`` / ``reverse_mapping``
dicts) and bit-for-bit the same strings of '0' / '1' characters.  The tree, code table, encoder and
decoder run in host C++ (csrc/huffman.cpp, tmae_huffman_*): the reference builds them in Python over
per-element ``int(value)`` loops.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib

_CAP = 1 << 16  # distinct values per table (ids_restore holds L <= a few hundred)


class HuffmanCoding:
    def __init__(self):
        self.heap = []
        self.codes = {}
        self.reverse_mapping = {}
        self._table = None

    # ---- tree + codes (build_heap / build_tree / build_codes, huffman.py:49-103)
    def build_codes_from(self, tensor):
        vals = np.ascontiguousarray(tensor.detach().reshape(-1).cpu().numpy().astype(np.int64))
        syms = np.empty(min(_CAP, max(1, vals.size)), dtype=np.int64)
        lens = np.empty_like(syms, dtype=np.int32)
        codes = np.empty_like(syms, dtype=np.uint64)
        n = ctypes.c_int(0)
        _lib.call("tmae_huffman_build", vals.ctypes.data, vals.size, syms.ctypes.data, lens.ctypes.data,
                  codes.ctypes.data, syms.size, ctypes.byref(n))
        k = n.value
        self._table = (syms[:k].copy(), lens[:k].copy(), codes[:k].copy())
        self.codes = {int(s): _bits(int(c), int(l)) for s, l, c in zip(*self._table)}
        self.reverse_mapping = {v: k_ for k_, v in self.codes.items()}
        return vals

    def encode(self, tensor):
        vals = np.ascontiguousarray(tensor.detach().reshape(-1).cpu().numpy().astype(np.int64))
        return self._encode(vals)

    def _encode(self, vals):
        syms, lens, codes = self._table
        nbits = ctypes.c_longlong(0)
        _lib.call("tmae_huffman_encode", vals.ctypes.data, vals.size, syms.ctypes.data, lens.ctypes.data,
                  codes.ctypes.data, syms.size, None, 0, ctypes.byref(nbits))
        buf = ctypes.create_string_buffer(max(1, nbits.value))
        _lib.call("tmae_huffman_encode", vals.ctypes.data, vals.size, syms.ctypes.data, lens.ctypes.data,
                  codes.ctypes.data, syms.size, buf, nbits.value, ctypes.byref(nbits))
        return buf.raw[:nbits.value].decode("ascii")

    def decode(self, encoded_text):
        syms, lens, codes = self._table
        raw = encoded_text.encode("ascii", errors="replace")
        out = np.empty(max(1, len(raw)), dtype=np.int64)
        n = ctypes.c_longlong(0)
        _lib.call("tmae_huffman_decode", raw, len(raw), syms.ctypes.data, lens.ctypes.data, codes.ctypes.data,
                  syms.size, out.ctypes.data, out.size, ctypes.byref(n))
        return torch.from_numpy(out[:n.value].copy())

    def compress(self, tensor):
        vals = self.build_codes_from(tensor)
        return self._encode(vals), tensor.shape, tensor.device

    def decompress(self, encoded_text, ori_shape, device):
        return self.decode(encoded_text).to(device).view(ori_shape)


def _bits(code, length):
    return format(code, "b").zfill(length) if length else ""
