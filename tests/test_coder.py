"""Host entropy coder (csrc/rans.cpp through textmae_amd.coder) against the pure-Python restatement
of compressai 1.2.4's coder (oracle/rans_oracle.py).  CPU only: the coder is host code.

compressai is not installed here and the reference holds no coded streams, so agreement with the
real package is **parity unpinned**; these tests pin the restatement bit-exactly and check
round trips, including the bypass escape for out-of-range values."""
import numpy as np
import pytest

from oracle import rans_oracle as ro


@pytest.fixture(scope="module")
def coder(tmae):
    from textmae_amd import coder as c

    return c


def random_pmf(rng, n, zeros=0):
    p = rng.random(n).astype(np.float64) ** 3
    if zeros:
        p[rng.choice(n, zeros, replace=False)] = 0.0
    p /= p.sum()
    return p.astype(np.float32)


@pytest.mark.parametrize("n,zeros", [(2, 0), (5, 0), (17, 3), (63, 20), (300, 150), (3000, 0)])
def test_pmf_to_quantized_cdf_matches_restatement(coder, n, zeros):
    rng = np.random.default_rng(n * 7 + zeros)
    pmf = random_pmf(rng, n, zeros)
    got = coder.pmf_to_quantized_cdf(pmf, 16)
    assert got == ro.pmf_to_quantized_cdf(pmf, 16)
    assert got[0] == 0 and got[-1] == 1 << 16 and all(b > a for a, b in zip(got, got[1:]))


def test_pmf_to_quantized_cdf_tail_mass(coder):
    """a Gaussian-like pmf with a tiny tail mass appended (EntropyModel._pmf_to_cdf)"""
    x = np.arange(-40, 41, dtype=np.float64)
    p = np.exp(-0.5 * (x / 6.0) ** 2)
    p = (p / p.sum() * (1 - 2e-9)).astype(np.float32)
    pmf = np.concatenate([p, np.float32([2e-9])])
    assert coder.pmf_to_quantized_cdf(pmf) == ro.pmf_to_quantized_cdf(pmf)


def test_pmf_to_quantized_cdf_rejects_bad_input(coder):
    with pytest.raises(ValueError, match="invalid pmf"):
        coder.pmf_to_quantized_cdf([0.5, -0.1, 0.6])
    with pytest.raises(ValueError, match="sums to 0"):
        coder.pmf_to_quantized_cdf([0.0, 0.0])


def tables(rng, ncdf, max_len=40):
    cdfs, sizes, offsets = [], [], []
    for _ in range(ncdf):
        n = int(rng.integers(2, max_len))
        cdf = ro.pmf_to_quantized_cdf(random_pmf(rng, n, zeros=int(rng.integers(0, n // 2 + 1))))
        cdfs.append(cdf)
        sizes.append(len(cdf))  # compressai: _cdf_length = pmf_length + 2 = entries incl. the tail bin
        offsets.append(int(rng.integers(-n, 1)))
    width = max(sizes)
    return [c + [0] * (width - len(c)) for c in cdfs], sizes, offsets


def symbols_for(rng, n, idx, sizes, offsets, escape_frac=0.05):
    out = []
    for ci in idx[:n]:
        lo, hi = offsets[ci], offsets[ci] + sizes[ci] - 2
        r = rng.random()
        if r < escape_frac / 2:
            out.append(int(lo - rng.integers(1, 1 << int(rng.integers(1, 20)))))   # below range
        elif r < escape_frac:
            out.append(int(hi + rng.integers(0, 1 << int(rng.integers(1, 20)))))   # at/above range
        else:
            out.append(int(rng.integers(lo, hi)))
    return out


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_stream_bit_exact_with_restatement(coder, seed):
    rng = np.random.default_rng(seed)
    cdfs, sizes, offsets = tables(rng, 12)
    idx = rng.integers(0, 12, 3000).tolist()
    sym = symbols_for(rng, 3000, idx, sizes, offsets)
    enc = coder.BufferedRansEncoder()
    enc.encode_with_indexes(sym[:1000], idx[:1000], cdfs, sizes, offsets)   # two calls = one stream
    enc.encode_with_indexes(sym[1000:], idx[1000:], cdfs, sizes, offsets)
    got = enc.flush()
    want = ro.encode(sym, idx, cdfs, sizes, offsets)
    assert got == want
    assert ro.Decoder(got).decode(idx, cdfs, sizes, offsets) == sym
    dec = coder.RansDecoder()
    dec.set_stream(got)
    parts = [dec.decode_stream(idx[a:b], cdfs, sizes, offsets) for a, b in ((0, 7), (7, 1500), (1500, 3000))]
    assert sum(parts, []) == sym


def test_extreme_escapes_round_trip(coder):
    cdfs = [[0, 30000, 65000, 65536]]
    sizes, offsets = [4], [0]
    sym = [0, 1, 2, 3, -1, -(1 << 30), (1 << 30), 17, -5, 2, 65535, -70000]
    enc = coder.RansEncoder().encode_with_indexes(sym, [0] * len(sym), cdfs, sizes, offsets)
    assert enc == ro.encode(sym, [0] * len(sym), cdfs, sizes, offsets)
    assert coder.RansDecoder().decode_with_indexes(enc, [0] * len(sym), cdfs, sizes, offsets) == sym


def test_large_round_trip_numpy_inputs(coder):
    rng = np.random.default_rng(5)
    cdfs, sizes, offsets = tables(rng, 64, max_len=200)
    n = 400_000
    idx = rng.integers(0, 64, n).astype(np.int32)
    lo = np.asarray(offsets)[idx]
    span = np.asarray(sizes)[idx] - 2
    sym = (lo + (rng.random(n) * span).astype(np.int32)).astype(np.int32)
    sym[::997] += 5000  # sprinkle escapes
    cdf_t = np.asarray(cdfs, dtype=np.int32)
    enc = coder.BufferedRansEncoder()
    enc.encode_with_indexes(sym, idx, cdf_t, sizes, offsets)
    s = enc.flush()
    dec = coder.RansDecoder()
    dec.set_stream(s)
    np.testing.assert_array_equal(dec.decode_stream_array(idx, cdf_t, sizes, offsets), sym)


def test_coder_errors(coder):
    cdfs, sizes, offsets = [[0, 1000, 65536, 0]], [3], [0]
    enc = coder.BufferedRansEncoder()
    with pytest.raises(ValueError, match="outside"):
        enc.encode_with_indexes([0], [1], cdfs, sizes, offsets)
    with pytest.raises(ValueError, match="cdf_sizes"):
        enc.encode_with_indexes([0], [0], cdfs, [9], offsets)
    with pytest.raises(ValueError, match="span"):
        enc.encode_with_indexes([0], [0], cdfs, [4], offsets)
    with pytest.raises(ValueError, match="strictly"):
        enc.encode_with_indexes([0], [0], [[0, 1000, 1000, 65536]], [4], offsets)
    with pytest.raises(ValueError, match="32-bit words"):
        coder.RansDecoder().set_stream(b"abc")
    s = coder.RansEncoder().encode_with_indexes([0, 1] * 50, [0] * 100, cdfs, sizes, offsets)
    dec = coder.RansDecoder()
    dec.set_stream(s[:8])
    with pytest.raises(ValueError, match="exhausted|corrupt"):
        dec.decode_stream([0] * 100, cdfs, sizes, offsets)
