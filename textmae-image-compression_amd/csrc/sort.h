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
