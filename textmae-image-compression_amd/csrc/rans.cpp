// Host-side entropy coder behind MCM.compress / decompress (reference MCM.py:845, 882-887,
// 917-918, 941-945 call compressai's BufferedRansEncoder / RansDecoder; testing.py:223 builds the
// CDF tables through EntropyBottleneck.update / GaussianConditional.update_scale_table).
//
// compressai 1.2.4 is a third-party dependency that is not vendored in the reference and not
// installed here; this is a restatement of its published coder so streams are interchangeable:
//   * 64-bit rANS state kept in [2^31, 2^63), 32-bit words written from the END of the buffer and
//     read back from the front, a final 8-byte state flush (ryg_rans "rans64" construction);
//   * 16-bit probability precision: symbol s of CDF c occupies [cdf[s], cdf[s+1]) of 2^16;
//   * values outside a CDF's range [offset, offset + size - 2) are escaped through its last symbol
//     (size - 2) followed by bypass nibbles: the nibble count as a run of 4-bit digits (15 = "more"),
//     then the raw value (negatives 2|v|-1, overflow 2(v - max)) 4 bits at a time, LSB first;
//   * the encoder buffers (start, freq, bypass) triples in coding order and writes them in reverse
//     at flush, so the decoder reads in forward order.
// The CDF builder restates compressai's pmf_to_quantized_cdf (round to 2^precision, rescale to the
// exact total, then steal one unit from the smallest >1 bin for every zero-width bin).
//
// Everything here is plain host code (no device work); handles are independent objects, so
// encoders/decoders on different threads do not interact.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <numeric>
#include <vector>

#include "tmae.h"

void tmae_set_error(int code, const char* fmt, ...);

#define RANS_REQUIRE(cond, ...)                 \
  do {                                          \
    if (!(cond)) {                              \
      tmae_set_error(TMAE_EINVAL, __VA_ARGS__); \
      return TMAE_EINVAL;                       \
    }                                           \
  } while (0)

namespace {

constexpr uint32_t kPrecision = 16;
constexpr uint32_t kBypassBits = 4;
constexpr uint32_t kBypassMax = (1u << kBypassBits) - 1;  // 15: "another nibble of count follows"
constexpr uint64_t kRansLow = 1ull << 31;                 // lower end of the normalised state interval

struct Sym {
  uint16_t start, freq;
  bool bypass;
};

struct Encoder {
  std::vector<Sym> syms;
  std::vector<uint8_t> bytes;  // result of the last flush
};

struct Decoder {
  std::vector<uint32_t> words;
  size_t pos = 0;
  uint64_t state = 0;
  bool overrun = false;

  uint32_t next_word() {
    if (pos >= words.size()) {
      overrun = true;
      return 0;
    }
    return words[pos++];
  }
  // pop `nbits` raw bits (bypass digits) and renormalise
  uint32_t get_bits(uint32_t nbits) {
    const uint32_t v = (uint32_t)(state & ((1ull << nbits) - 1));
    state >>= nbits;
    if (state < kRansLow) state = (state << 32) | next_word();
    return v;
  }
  uint32_t peek(uint32_t scale_bits) const { return (uint32_t)(state & ((1ull << scale_bits) - 1)); }
  void advance(uint32_t start, uint32_t freq, uint32_t scale_bits) {
    const uint64_t mask = (1ull << scale_bits) - 1;
    state = (uint64_t)freq * (state >> scale_bits) + (state & mask) - start;
    if (state < kRansLow) state = (state << 32) | next_word();
  }
};

// rANS encode step (C(s, x)) with output renormalisation; `out` grows downward
inline void enc_put(uint64_t& x, std::vector<uint32_t>& out, size_t& head, uint32_t start, uint32_t freq,
                    uint32_t scale_bits) {
  const uint64_t x_max = ((kRansLow >> scale_bits) << 32) * freq;
  if (x >= x_max) {
    out[--head] = (uint32_t)x;
    x >>= 32;
  }
  x = ((x / freq) << scale_bits) + (x % freq) + start;
}

// raw bits: same interval arithmetic with freq = 2^(16 - nbits) of a 2^16 range
inline void enc_put_bits(uint64_t& x, std::vector<uint32_t>& out, size_t& head, uint32_t val, uint32_t nbits) {
  const uint32_t freq = 1u << (kPrecision - nbits);
  const uint64_t x_max = ((kRansLow >> kPrecision) << 32) * freq;
  if (x >= x_max) {
    out[--head] = (uint32_t)x;
    x >>= 32;
  }
  x = (x << nbits) | val;
}

int check_tables(const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes, const int32_t* offsets, int ncdf) {
  RANS_REQUIRE(cdfs && cdf_sizes && offsets && ncdf > 0 && cdf_stride > 1, "rans: CDF tables required");
  for (int c = 0; c < ncdf; ++c) {
    const int32_t n = cdf_sizes[c];
    RANS_REQUIRE(n >= 3 && n <= cdf_stride, "rans: cdf_sizes[%d] = %d outside [3, %d]", c, n, cdf_stride);
    // a malformed table must fail here, not as a zero-width symbol (division by zero) while coding
    const int32_t* cdf = cdfs + (size_t)c * cdf_stride;
    RANS_REQUIRE(cdf[0] == 0 && cdf[n - 1] == (1 << kPrecision), "rans: cdf %d does not span [0, 2^%u]", c, kPrecision);
    for (int32_t i = 1; i < n; ++i)
      RANS_REQUIRE(cdf[i] > cdf[i - 1], "rans: cdf %d is not strictly increasing at %d", c, i);
  }
  (void)offsets;
  return TMAE_OK;
}

}  // namespace

// ------------------------------------------------------------------ CDF construction
extern "C" int tmae_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int32_t* cdf_out) {
  RANS_REQUIRE(pmf && cdf_out && n > 0 && precision > 0 && precision <= 16, "tmae_pmf_to_quantized_cdf: bad arguments");
  for (int i = 0; i < n; ++i)
    RANS_REQUIRE(pmf[i] >= 0.0f && std::isfinite(pmf[i]), "tmae_pmf_to_quantized_cdf: invalid pmf[%d] = %g", i,
                 (double)pmf[i]);
  const uint32_t one = 1u << precision;
  std::vector<uint32_t> cdf(n + 1);
  cdf[0] = 0;
  for (int i = 0; i < n; ++i) cdf[i + 1] = (uint32_t)std::round(pmf[i] * (float)one);
  uint32_t total = 0;
  for (uint32_t v : cdf) total += v;
  RANS_REQUIRE(total != 0, "tmae_pmf_to_quantized_cdf: pmf sums to 0 at precision %d", precision);
  for (uint32_t& v : cdf) v = (uint32_t)(((uint64_t)one * v) / total);
  std::partial_sum(cdf.begin(), cdf.end(), cdf.begin());
  cdf.back() = one;
  // every symbol needs a non-empty interval: take one unit from the smallest bin that can spare it
  for (int i = 0; i < n; ++i) {
    if (cdf[i] != cdf[i + 1]) continue;
    uint32_t best = ~0u;
    int steal = -1;
    for (int j = 0; j < n; ++j) {
      const uint32_t f = cdf[j + 1] - cdf[j];
      if (f > 1 && f < best) {
        best = f;
        steal = j;
      }
    }
    RANS_REQUIRE(steal >= 0, "tmae_pmf_to_quantized_cdf: no bin to steal from (n=%d)", n);
    if (steal < i) {
      for (int j = steal + 1; j <= i; ++j) cdf[j]--;
    } else {
      for (int j = i + 1; j <= steal; ++j) cdf[j]++;
    }
  }
  for (int i = 0; i <= n; ++i) cdf_out[i] = (int32_t)cdf[i];
  return TMAE_OK;
}

// ------------------------------------------------------------------ encoder
extern "C" int tmae_rans_encoder_create(void** handle) {
  RANS_REQUIRE(handle != nullptr, "tmae_rans_encoder_create: handle is NULL");
  *handle = new (std::nothrow) Encoder();
  RANS_REQUIRE(*handle != nullptr, "tmae_rans_encoder_create: out of memory");
  return TMAE_OK;
}

extern "C" int tmae_rans_encoder_destroy(void* handle) {
  delete static_cast<Encoder*>(handle);
  return TMAE_OK;
}

// BufferedRansEncoder.encode_with_indexes: symbol i is coded with CDF indexes[i]
extern "C" int tmae_rans_encode_with_indexes(void* handle, const int32_t* symbols, const int32_t* indexes,
                                             long long n, const int32_t* cdfs, int cdf_stride,
                                             const int32_t* cdf_sizes, const int32_t* offsets, int ncdf) {
  RANS_REQUIRE(handle != nullptr && n >= 0 && (n == 0 || (symbols && indexes)), "tmae_rans_encode_with_indexes: bad arguments");
  if (int rc = check_tables(cdfs, cdf_stride, cdf_sizes, offsets, ncdf)) return rc;
  Encoder* e = static_cast<Encoder*>(handle);
  e->syms.reserve(e->syms.size() + (size_t)n);
  for (long long i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    RANS_REQUIRE(ci >= 0 && ci < ncdf, "tmae_rans_encode_with_indexes: index[%lld] = %d outside [0, %d)", i, ci, ncdf);
    const int32_t* cdf = cdfs + (size_t)ci * cdf_stride;
    const int32_t max_value = cdf_sizes[ci] - 2;
    int32_t value = symbols[i] - offsets[ci];
    uint32_t raw = 0;
    if (value < 0) {
      raw = (uint32_t)(-2 * (int64_t)value - 1);
      value = max_value;
    } else if (value >= max_value) {
      raw = (uint32_t)(2 * (int64_t)(value - max_value));
      value = max_value;
    }
    e->syms.push_back({(uint16_t)cdf[value], (uint16_t)(cdf[value + 1] - cdf[value]), false});
    if (value != max_value) continue;
    // escape: count of 4-bit digits of `raw`, then the digits
    uint32_t ndig = 0;
    while (ndig < 8 && (raw >> (ndig * kBypassBits)) != 0) ++ndig;
    uint32_t cnt = ndig;
    while (cnt >= kBypassMax) {
      e->syms.push_back({(uint16_t)kBypassMax, (uint16_t)(kBypassMax + 1), true});
      cnt -= kBypassMax;
    }
    e->syms.push_back({(uint16_t)cnt, (uint16_t)(cnt + 1), true});
    for (uint32_t d = 0; d < ndig; ++d) {
      const uint32_t v = (raw >> (d * kBypassBits)) & kBypassMax;
      e->syms.push_back({(uint16_t)v, (uint16_t)(v + 1), true});
    }
  }
  return TMAE_OK;
}

// BufferedRansEncoder.flush: code the buffered symbols (last first) into one stream; the encoder is
// empty afterwards.  *nbytes = stream length; fetch it with tmae_rans_encoder_take.
extern "C" int tmae_rans_encoder_flush(void* handle, long long* nbytes) {
  RANS_REQUIRE(handle != nullptr && nbytes != nullptr, "tmae_rans_encoder_flush: bad arguments");
  Encoder* e = static_cast<Encoder*>(handle);
  std::vector<uint32_t> out(e->syms.size() + 2);
  size_t head = out.size();
  uint64_t x = kRansLow;
  for (size_t k = e->syms.size(); k-- > 0;) {
    const Sym& s = e->syms[k];
    if (s.bypass) enc_put_bits(x, out, head, s.start, kBypassBits);
    else enc_put(x, out, head, s.start, s.freq, kPrecision);
  }
  out[--head] = (uint32_t)(x >> 32);
  out[--head] = (uint32_t)x;
  // little-endian 32-bit words in stream order
  const size_t words = out.size() - head;
  e->bytes.resize(words * 4);
  memcpy(e->bytes.data(), out.data() + head, words * 4);
  e->syms.clear();
  *nbytes = (long long)e->bytes.size();
  return TMAE_OK;
}

extern "C" int tmae_rans_encoder_take(void* handle, uint8_t* out, long long cap) {
  RANS_REQUIRE(handle != nullptr, "tmae_rans_encoder_take: handle is NULL");
  Encoder* e = static_cast<Encoder*>(handle);
  RANS_REQUIRE(out != nullptr && cap >= (long long)e->bytes.size(), "tmae_rans_encoder_take: buffer of %lld < %lld bytes",
               cap, (long long)e->bytes.size());
  memcpy(out, e->bytes.data(), e->bytes.size());
  e->bytes.clear();
  return TMAE_OK;
}

// ------------------------------------------------------------------ decoder
// RansDecoder.set_stream: the stream is copied, so the caller's buffer may go away
extern "C" int tmae_rans_decoder_create(const uint8_t* data, long long len, void** handle) {
  RANS_REQUIRE(handle != nullptr && data != nullptr && len >= 8 && len % 4 == 0,
               "tmae_rans_decoder_create: a stream is a whole number of 32-bit words, >= 8 bytes (got %lld)", len);
  Decoder* d = new (std::nothrow) Decoder();
  RANS_REQUIRE(d != nullptr, "tmae_rans_decoder_create: out of memory");
  d->words.resize((size_t)len / 4);
  memcpy(d->words.data(), data, (size_t)len);
  const uint64_t lo = d->next_word(), hi = d->next_word();
  d->state = lo | (hi << 32);
  *handle = d;
  return TMAE_OK;
}

extern "C" int tmae_rans_decoder_destroy(void* handle) {
  delete static_cast<Decoder*>(handle);
  return TMAE_OK;
}

// RansDecoder.decode_stream: the next n symbols of the stream, symbol i with CDF indexes[i]
extern "C" int tmae_rans_decode_with_indexes(void* handle, const int32_t* indexes, long long n, const int32_t* cdfs,
                                             int cdf_stride, const int32_t* cdf_sizes, const int32_t* offsets,
                                             int ncdf, int32_t* out) {
  RANS_REQUIRE(handle != nullptr && n >= 0 && (n == 0 || (indexes && out)), "tmae_rans_decode_with_indexes: bad arguments");
  if (int rc = check_tables(cdfs, cdf_stride, cdf_sizes, offsets, ncdf)) return rc;
  Decoder* d = static_cast<Decoder*>(handle);
  for (long long i = 0; i < n; ++i) {
    const int32_t ci = indexes[i];
    RANS_REQUIRE(ci >= 0 && ci < ncdf, "tmae_rans_decode_with_indexes: index[%lld] = %d outside [0, %d)", i, ci, ncdf);
    const int32_t* cdf = cdfs + (size_t)ci * cdf_stride;
    const int32_t size = cdf_sizes[ci];
    const int32_t max_value = size - 2;
    const uint32_t cum = d->peek(kPrecision);
    // symbol = last s with cdf[s] <= cum (cdf strictly increasing over [0, size))
    const int32_t* it = std::upper_bound(cdf, cdf + size, (int32_t)cum);
    const int32_t s = (int32_t)(it - cdf) - 1;
    RANS_REQUIRE(s >= 0 && s < size - 1, "tmae_rans_decode_with_indexes: corrupt stream at symbol %lld", i);
    d->advance((uint32_t)cdf[s], (uint32_t)(cdf[s + 1] - cdf[s]), kPrecision);
    int32_t value = s;
    if (value == max_value) {
      uint32_t v = d->get_bits(kBypassBits);
      uint32_t ndig = v;
      while (v == kBypassMax) {
        v = d->get_bits(kBypassBits);
        ndig += v;
      }
      RANS_REQUIRE(ndig <= 8, "tmae_rans_decode_with_indexes: corrupt escape at symbol %lld", i);
      uint32_t raw = 0;
      for (uint32_t k = 0; k < ndig; ++k) raw |= d->get_bits(kBypassBits) << (k * kBypassBits);
      const int32_t half = (int32_t)(raw >> 1);
      value = (raw & 1) ? -half - 1 : half + max_value;
    }
    RANS_REQUIRE(!d->overrun, "tmae_rans_decode_with_indexes: stream exhausted at symbol %lld", i);
    out[i] = value + offsets[ci];
  }
  return TMAE_OK;
}
