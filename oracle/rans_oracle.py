"""TEST INFRASTRUCTURE ONLY -- pure-Python restatement of compressai 1.2.4's entropy coder, the
checker for csrc/rans.cpp.  Imported only by tests/ (never by the product).

compressai is the reference's third-party dependency (requirements.txt:9; BufferedRansEncoder /
RansDecoder at models/Compression/MCM.py:845, 882-887, 890, 917-918, 941-945; pmf_to_quantized_cdf
via EntropyModel.update at testing.py:223).  It is neither vendored in /root/reference nor
installed here, so this restates its published algorithm (compressai/cpp_exts/rans/
rans_interface.cpp and ops.cpp on top of ryg_rans' rans64.h) -- **parity unpinned** against the real
package; round trips and bit-exact agreement with this restatement are what tests check.
"""
from __future__ import annotations

import math
import struct

import numpy as np

PRECISION = 16
BYPASS_BITS = 4
BYPASS_MAX = (1 << BYPASS_BITS) - 1
RANS_L = 1 << 31
M64 = (1 << 64) - 1


def pmf_to_quantized_cdf(pmf, precision=PRECISION):
    """ops.cpp pmf_to_quantized_cdf: std::round(p * 2^prec) in float32, rescale by the total,
    prefix sum, last = 2^prec, then give every empty bin one unit from the smallest bin > 1."""
    one = 1 << precision
    p32 = np.asarray(pmf, dtype=np.float32)
    cdf = [0] + [int(round_half_away(float(np.float32(v) * np.float32(one)))) for v in p32]
    total = sum(cdf)
    cdf = [(one * v) // total for v in cdf]
    for i in range(1, len(cdf)):
        cdf[i] += cdf[i - 1]
    cdf[-1] = one
    n = len(cdf) - 1
    for i in range(n):
        if cdf[i] != cdf[i + 1]:
            continue
        best, steal = None, -1
        for j in range(n):
            f = cdf[j + 1] - cdf[j]
            if f > 1 and (best is None or f < best):
                best, steal = f, j
        assert steal >= 0
        if steal < i:
            for j in range(steal + 1, i + 1):
                cdf[j] -= 1
        else:
            for j in range(i + 1, steal + 1):
                cdf[j] += 1
    return cdf


def round_half_away(x):
    """std::round (half away from zero)"""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def _escape(raw):
    ndig = 0
    while ndig < 8 and (raw >> (ndig * BYPASS_BITS)) != 0:
        ndig += 1
    out = []
    cnt = ndig
    while cnt >= BYPASS_MAX:
        out.append(BYPASS_MAX)
        cnt -= BYPASS_MAX
    out.append(cnt)
    out += [(raw >> (d * BYPASS_BITS)) & BYPASS_MAX for d in range(ndig)]
    return out


def encode(symbols, indexes, cdfs, cdf_sizes, offsets):
    """BufferedRansEncoder.encode_with_indexes + flush -> bytes"""
    syms = []  # (start, freq) or ("bits", value)
    for s, ci in zip(symbols, indexes):
        cdf = cdfs[ci]
        max_value = cdf_sizes[ci] - 2
        value = s - offsets[ci]
        raw = 0
        if value < 0:
            raw = -2 * value - 1
            value = max_value
        elif value >= max_value:
            raw = 2 * (value - max_value)
            value = max_value
        syms.append((cdf[value], cdf[value + 1] - cdf[value]))
        if value == max_value:
            syms += [("bits", v) for v in _escape(raw)]
    words = []  # emitted back to front
    x = RANS_L
    for sym in reversed(syms):
        if sym[0] == "bits":
            freq = 1 << (PRECISION - BYPASS_BITS)
            x_max = ((RANS_L >> PRECISION) << 32) * freq
            if x >= x_max:
                words.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x << BYPASS_BITS) | sym[1]) & M64
        else:
            start, freq = sym
            x_max = ((RANS_L >> PRECISION) << 32) * freq
            if x >= x_max:
                words.append(x & 0xFFFFFFFF)
                x >>= 32
            x = ((x // freq) << PRECISION) + (x % freq) + start
    words += [x >> 32, x & 0xFFFFFFFF]
    words.reverse()
    return struct.pack(f"<{len(words)}I", *words)


class Decoder:
    """RansDecoder.set_stream + decode_stream"""

    def __init__(self, data: bytes):
        self.w = list(struct.unpack(f"<{len(data) // 4}I", data))
        self.pos = 2
        self.x = self.w[0] | (self.w[1] << 32)

    def _renorm(self):
        if self.x < RANS_L:
            self.x = (self.x << 32) | self.w[self.pos]
            self.pos += 1

    def _bits(self, n):
        v = self.x & ((1 << n) - 1)
        self.x >>= n
        self._renorm()
        return v

    def decode(self, indexes, cdfs, cdf_sizes, offsets):
        out = []
        for ci in indexes:
            cdf, size = cdfs[ci], cdf_sizes[ci]
            max_value = size - 2
            cum = self.x & ((1 << PRECISION) - 1)
            s = max(j for j in range(size) if cdf[j] <= cum)
            start, freq = cdf[s], cdf[s + 1] - cdf[s]
            self.x = freq * (self.x >> PRECISION) + (self.x & ((1 << PRECISION) - 1)) - start
            self._renorm()
            value = s
            if value == max_value:
                v = self._bits(BYPASS_BITS)
                ndig = v
                while v == BYPASS_MAX:
                    v = self._bits(BYPASS_BITS)
                    ndig += v
                raw = 0
                for d in range(ndig):
                    raw |= self._bits(BYPASS_BITS) << (d * BYPASS_BITS)
                value = -(raw >> 1) - 1 if raw & 1 else (raw >> 1) + max_value
            out.append(value + offsets[ci])
        return out
