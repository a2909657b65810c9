// LDS sort helpers shared by the per-row index kernels (ids_shuffle.hip, mae.hip).
#pragma once

#include "common.h"

// order-preserving float -> uint map (negative values flipped), so (key << 32 | index) sorts by
// value, then index: a stable ascending argsort
__device__ __forceinline__ unsigned f2key(float f) {
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(unsigned k) {
  unsigned u = (k & 0x80000000u) ? (k & 0x7fffffffu) : ~k;
  return __uint_as_float(u);
}

// ascending bitonic sort of P (power of two) 64-bit keys in LDS by the whole workgroup
template <int NT>
__device__ __forceinline__ void lds_bitonic_sort(unsigned long long* key, int P) {
  const int t = threadIdx.x;
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < P; i += NT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = key[i], c = key[ixj];
          const bool up = ((i & k) == 0);
          if ((a > c) == up) { key[i] = c; key[ixj] = a; }
        }
      }
      __syncthreads();
    }
  }
}

// the same sort with one key per thread (P <= NT): the compare-exchange stages whose partner lies in the same
// wave (j < 64) run on registers through lane shuffles -- no LDS round trip, no workgroup barrier -- and only the
// j >= 64 stages go through LDS (two barriers each); 36 -> 3 barriered stages at P = 256.  The network and hence
// the result are the lds_bitonic_sort ones (the keys are distinct).  Leaves the sorted keys in key[0..P).
template <int NT>
__device__ __forceinline__ void reg_bitonic_sort(unsigned long long* key, int P) {
  const int t = threadIdx.x;
  unsigned long long v = t < P ? key[t] : ~0ull;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      unsigned long long w;
      if (j < 64) {
        const unsigned lo = __shfl_xor((unsigned)v, j, 64), hi = __shfl_xor((unsigned)(v >> 32), j, 64);
        w = ((unsigned long long)hi << 32) | lo;
      } else {
        key[t] = v;
        __syncthreads();
        w = key[t ^ j];
        __syncthreads();
      }
      const bool up = (t & k) == 0, lower = (t & j) == 0;
      const unsigned long long mn = v < w ? v : w, mx = v < w ? w : v;
      v = (lower == up) ? mn : mx;
    }
  }
  if (t < P) key[t] = v;
  __syncthreads();
}
