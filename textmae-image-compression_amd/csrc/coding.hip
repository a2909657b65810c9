// Device side of MCM.compress / decompress (reference MCM.py:805-968) around the host rANS coder
// (rans.cpp): the GaussianConditional CDF-table pmf (update_scale_table, testing.py:223), scale-table
// indexes (build_indexes, MCM.py:867, 938), dequantisation of decoded symbols into the slice loop's
// y_hat buffers (MCM.py:946), and the ids_restore -> ids_shuffle inverse the decoder kernels index by.
// The symbol-emitting form of the slice likelihood kernel lives with it in conv.hip
// (tmae_gc_slices_code); the EntropyBottleneck ones with its density tables in entropy.hip.
#include "common.h"

// GaussianConditional.update: pmf[i][j] = Phi((1/2 - s) / scale_i) - Phi((-1/2 - s) / scale_i),
// s = |j - center_i|, Phi(x) = erfc(-x / sqrt 2) / 2; tail[i] = 2 Phi((-1/2 - center_i) / scale_i)
__device__ __forceinline__ float std_cumulative(float x) { return 0.5f * erfcf(-0.70710678118654752440f * x); }

__global__ void __launch_bounds__(256)
gc_pmf_kernel(const float* __restrict__ scale_table, const int* __restrict__ center, int n, int max_length,
              float* __restrict__ pmf, float* __restrict__ tail) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * max_length) return;
  const int r = i / max_length, j = i - r * max_length;
  const float sc = scale_table[r];
  const float s = (float)abs(j - center[r]);
  const float upper = std_cumulative((0.5f - s) / sc);
  const float lower = std_cumulative((-0.5f - s) / sc);
  pmf[i] = upper - lower;
  if (j == 0) tail[r] = 2.0f * lower;
}

extern "C" int tmae_gc_pmf(const float* scale_table, const int* pmf_center, int n, int max_length, float* pmf,
                           float* tail, void* stream) {
  TMAE_REQUIRE(scale_table && pmf_center && pmf && tail && n > 0 && max_length > 0, "tmae_gc_pmf: bad arguments");
  hipLaunchKernelGGL(gc_pmf_kernel, dim3(ceil_div(n * max_length, 256)), dim3(256), 0, (hipStream_t)stream,
                     scale_table, pmf_center, n, max_length, pmf, tail);
  TMAE_LAUNCH_CHECK("tmae_gc_pmf");
}

// build_indexes: index = (nscale - 1) - #{t < nscale - 1 : max(sigma, bound) <= table[t]}.
// sigma rows: slice j of the launch at sigma + j * ms_stride, row m (= image * HW + pixel), channel c
// at m * ld_ms + c; indexes written in the coder's order [slice][image][channel][pixel].
__global__ void __launch_bounds__(256)
gc_indexes_kernel(const float* __restrict__ sigma, long long ms_stride, int ld_ms, int n, int HW, int nslices, int sw,
                  const float* __restrict__ scale_table, int nscale, float bound, int* __restrict__ idx, int total) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int per_pix = nslices * sw;
  const int m = i / per_pix, r = i - m * per_pix;
  const int j = r / sw, c = r - j * sw;
  const int b = m / HW, pix = m - b * HW;
  const float s = fmaxf(sigma[j * ms_stride + (size_t)m * ld_ms + c], bound);
  int id = nscale - 1;
  for (int t = 0; t < nscale - 1; ++t) id -= (s <= scale_table[t]) ? 1 : 0;
  idx[(size_t)j * n * sw * HW + ((size_t)b * sw + c) * HW + pix] = id;
}

extern "C" int tmae_gc_indexes(const float* sigma, long long ms_stride, int ld_ms, int n, int HW, int nslices, int sw,
                               const float* scale_table, int nscale, float scale_bound, int* indexes, void* stream) {
  TMAE_REQUIRE(sigma && scale_table && indexes && nscale >= 1, "tmae_gc_indexes: bad arguments");
  const int total = n * HW * nslices * sw;
  if (total <= 0) return TMAE_OK;
  hipLaunchKernelGGL(gc_indexes_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, sigma,
                     ms_stride, ld_ms, n, HW, nslices, sw, scale_table, nscale, scale_bound, indexes, total);
  TMAE_LAUNCH_CHECK("tmae_gc_indexes");
}

// decompress: y_hat_pre = symbols + mu (GaussianConditional.dequantize, MCM.py:946) into the same
// slice buffers the forward's slice kernel writes (operand dtype + f32 copy for the LRP residual)
template <typename YT>
__global__ void __launch_bounds__(256)
gc_dequantize_kernel(const int* __restrict__ sym, const float* __restrict__ mu, long long ms_stride, int ld_ms, int n,
                     int HW, int nslices, int sw, int yoff, YT* __restrict__ yhat, int ld_yhat,
                     float* __restrict__ yhat32, int ld32, int total) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int per_pix = nslices * sw;
  const int m = i / per_pix, r = i - m * per_pix;
  const int j = r / sw, c = r - j * sw;
  const int b = m / HW, pix = m - b * HW;
  const int ch = yoff + j * sw + c;
  const float q = (float)sym[(size_t)j * n * sw * HW + ((size_t)b * sw + c) * HW + pix] +
                  mu[j * ms_stride + (size_t)m * ld_ms + c];
  yhat[(size_t)m * ld_yhat + ch] = to_out<YT>(q);
  if (yhat32) yhat32[(size_t)m * ld32 + ch] = q;
}

extern "C" int tmae_gc_dequantize(const int* symbols, const float* mu, long long ms_stride, int ld_ms, int n, int HW,
                                  int nslices, int sw, int yoff, void* yhat, int yhat_dtype, int ld_yhat,
                                  float* yhat32, int ld32, void* stream) {
  TMAE_REQUIRE(symbols && mu && yhat, "tmae_gc_dequantize: bad arguments");
  const int total = n * HW * nslices * sw;
  if (total <= 0) return TMAE_OK;
  const dim3 grid(ceil_div(total, 256));
  if (yhat_dtype == TMAE_BF16)
    hipLaunchKernelGGL(gc_dequantize_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, symbols, mu, ms_stride,
                       ld_ms, n, HW, nslices, sw, yoff, (bf16*)yhat, ld_yhat, yhat32, ld32, total);
  else
    hipLaunchKernelGGL(gc_dequantize_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, symbols, mu, ms_stride,
                       ld_ms, n, HW, nslices, sw, yoff, (float*)yhat, ld_yhat, yhat32, ld32, total);
  TMAE_LAUNCH_CHECK("tmae_gc_dequantize");
}

// inv[b][p[b][j]] = j  (ids_shuffle = argsort(ids_restore) for a permutation, MCM.py:580)
__global__ void invert_permutation_kernel(const int64_t* __restrict__ p, int64_t* __restrict__ inv, int L, int total) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int b = i / L, j = i - b * L;
  const int64_t v = p[i];
  if (v >= 0 && v < L) inv[(size_t)b * L + v] = j;
}

extern "C" int tmae_invert_permutation(const int64_t* perm, int64_t* inverse, int n, int L, void* stream) {
  TMAE_REQUIRE(perm && inverse && n >= 0 && L >= 0, "tmae_invert_permutation: bad arguments");
  const int total = n * L;
  if (total <= 0) return TMAE_OK;
  hipLaunchKernelGGL(invert_permutation_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, perm,
                     inverse, L, total);
  TMAE_LAUNCH_CHECK("tmae_invert_permutation");
}
