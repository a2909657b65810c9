// Entropy-model kernels (compressai 1.2.4 semantics; the package is not vendored in the reference,
// call sites MCM.py:71-72, 741-744, 771-776, utils/engine.py:79).
//
//  * EntropyBottleneck: per-channel monotone density MLP 1-3-3-3-3-1 (_logits_cumulative),
//    likelihood |sigmoid(s*f(x+1/2)) - sigmoid(s*f(x-1/2))|, s = -sign(f(x+1/2) + f(x-1/2)),
//    LowerBound(1e-9).  Input x = round(z - median) + median (eval) or z + U(-1/2, 1/2) (train).
//    The parameter transforms softplus(matrix) / tanh(factor) are computed once per channel into a
//    packed 59-float table (prep kernel), then one thread per latent element: memory-bound, coalesced
//    over the NHWC z tensor.
//  * GaussianConditional likelihood (standalone form; the slice loop uses the fused conv epilogue
//    in gemm.hip).
//  * aux_loss = sum |f(quantiles) - target|.
#include "common.h"

#define EB_PACK 59

__device__ __forceinline__ float softplus_t(float x) {  // F.softplus(beta=1, threshold=20)
  return x > 20.0f ? x : log1pf(expf(x));
}
__device__ __forceinline__ float sigmoid_t(float x) { return 1.0f / (1.0f + expf(-x)); }

// per-channel parameter table [C][EB_PACK]: softplus(matrices), biases, tanh(factors), median.
// One thread per table element (the table is tiny; a thread per channel walking 59 strided loads
// was latency-bound at ~26 us).
__global__ void __launch_bounds__(256) eb_prep_kernel(tmae_eb_params p, float* __restrict__ tab, int C) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * EB_PACK) return;
  const int c = i / EB_PACK, e = i - c * EB_PACK;
  float v;
  if (e < 9) {  // layer 0: matrix [C][3][1], bias [C][3][1], factor [C][3][1]
    const int g = e / 3, j = e - 3 * g;
    v = g == 0 ? softplus_t(p.matrix[0][c * 3 + j]) : g == 1 ? p.bias[0][c * 3 + j] : tanhf(p.factor[0][c * 3 + j]);
  } else if (e < 54) {  // layers 1..3: matrix [C][3][3], bias [C][3][1], factor [C][3][1]
    const int l = 1 + (e - 9) / 15, q = (e - 9) % 15;
    v = q < 9 ? softplus_t(p.matrix[l][c * 9 + q])
              : q < 12 ? p.bias[l][c * 3 + (q - 9)] : tanhf(p.factor[l][c * 3 + (q - 12)]);
  } else if (e < 57) {  // layer 4: matrix [C][1][3]
    v = softplus_t(p.matrix[4][c * 3 + (e - 54)]);
  } else if (e == 57) {
    v = p.bias[4][c];
  } else {
    v = p.quantiles[c * 3 + 1];  // _get_medians(): quantiles[:, :, 1:2]
  }
  tab[i] = v;
}

__device__ __forceinline__ float eb_logits(const float* t, float v) {
  float h0 = t[0] * v + t[3], h1 = t[1] * v + t[4], h2 = t[2] * v + t[5];
  h0 += t[6] * tanhf(h0);
  h1 += t[7] * tanhf(h1);
  h2 += t[8] * tanhf(h2);
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const float* q = t + 9 + 15 * l;
    float g0 = (q[0] * h0 + q[1] * h1 + q[2] * h2) + q[9];
    float g1 = (q[3] * h0 + q[4] * h1 + q[5] * h2) + q[10];
    float g2 = (q[6] * h0 + q[7] * h1 + q[8] * h2) + q[11];
    g0 += q[12] * tanhf(g0);
    g1 += q[13] * tanhf(g1);
    g2 += q[14] * tanhf(g2);
    h0 = g0; h1 = g1; h2 = g2;
  }
  return (t[54] * h0 + t[55] * h1 + t[56] * h2) + t[57];
}

// z, zhat: NHWC [n*HW][C]; lik, noise: NCHW [n][C][HW].
// One workgroup per (image, 64-channel block): element e = pix * 64 + c, so z / zhat are read / written in 256-B
// channel runs, and the block's lik (and noise) region [b][c0 .. c0 + 63][0 .. HW) is one contiguous NCHW range
// written by this workgroup alone.  (One thread per NHWC element, as before round 5, wrote each NCHW line from ~HW
// workgroups on different XCDs at a 4 * HW-B stride: PMC 1.93x the algorithmic bytes.)
__global__ void __launch_bounds__(256)
eb_likelihood_kernel(const float* __restrict__ z, const float* __restrict__ tab, const float* __restrict__ noise,
                     float* __restrict__ lik, void* __restrict__ zhat, int zhat_bf16, int C, int HW) {
  const int nblk = (C + 63) >> 6;
  const int b = blockIdx.x / nblk, c0 = (blockIdx.x - b * nblk) * 64;
  for (int e = threadIdx.x; e < 64 * HW; e += 256) {
    const int pix = e >> 6, c = c0 + (e & 63);
    if (c >= C) continue;
    const size_t i = ((size_t)b * HW + pix) * C + c;
    const float* t = tab + (size_t)c * EB_PACK;
    const float med = t[58];
    const float zv = z[i];
    const float q = rintf(zv - med) + med;
    const size_t nchw = ((size_t)b * C + c) * HW + pix;
    const float x = noise ? zv + noise[nchw] : q;
    const float lower = eb_logits(t, x - 0.5f);
    const float upper = eb_logits(t, x + 0.5f);
    const float sum = lower + upper;
    const float sgn = sum > 0.0f ? -1.0f : (sum < 0.0f ? 1.0f : -0.0f);
    const float l = fabsf(sigmoid_t(sgn * upper) - sigmoid_t(sgn * lower));
    lik[nchw] = fmaxf(l, 1e-9f);
    // quantize_ste forward value: round(z - med) + med  (MCM.py:742-744)
    if (zhat) {
      if (zhat_bf16) ((bf16*)zhat)[i] = (bf16)q;
      else ((float*)zhat)[i] = q;
    }
  }
}

extern "C" int tmae_eb_likelihood_fwd(const float* z, const tmae_eb_params* params, const float* noise, float* lik,
                                      void* zhat, int zhat_dtype, float* table, int n, int C, int HW, void* stream) {
  TMAE_REQUIRE(params != nullptr && table != nullptr, "tmae_eb_likelihood_fwd: params/table required");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(eb_prep_kernel, dim3(ceil_div(C * EB_PACK, 256)), dim3(256), 0, st, *params, table, C);
  const long long total = (long long)n * HW * C;
  if (total > 0) {
    TMAE_REQUIRE(total < (1ll << 31), "tmae_eb_likelihood_fwd: %lld elements exceed the 32-bit range", total);
    hipLaunchKernelGGL(eb_likelihood_kernel, dim3(n * ceil_div(C, 64)), dim3(256), 0, st, z, table, noise, lik, zhat,
                       zhat_dtype == TMAE_BF16, C, HW);
  }
  TMAE_LAUNCH_CHECK("tmae_eb_likelihood_fwd");
}

// aux loss: sum_c sum_j |f_c(quantiles[c][j]) - target[j]|   (compressai EntropyBottleneck.loss)
__global__ void __launch_bounds__(256)
eb_aux_loss_kernel(const float* __restrict__ tab, const float* __restrict__ quantiles,
                   const float* __restrict__ target, float* __restrict__ out, int C) {
  __shared__ float red[256];
  float s = 0.0f;
  for (int i = threadIdx.x; i < C * 3; i += 256) {
    const int c = i / 3, j = i - 3 * c;
    s += fabsf(eb_logits(tab + (size_t)c * EB_PACK, quantiles[i]) - target[j]);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

extern "C" int tmae_eb_aux_loss(const tmae_eb_params* params, const float* target, float* out, float* table, int C,
                                void* stream) {
  TMAE_REQUIRE(params != nullptr && table != nullptr, "tmae_eb_aux_loss: params/table required");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(eb_prep_kernel, dim3(ceil_div(C * EB_PACK, 256)), dim3(256), 0, st, *params, table, C);
  hipLaunchKernelGGL(eb_aux_loss_kernel, dim3(1), dim3(256), 0, st, table, params->quantiles, target, out, C);
  TMAE_LAUNCH_CHECK("tmae_eb_aux_loss");
}

// GaussianConditional.forward (elementwise, identical layouts): outputs y~ and likelihood
__global__ void __launch_bounds__(256)
gc_likelihood_kernel(const float* __restrict__ x, const float* __restrict__ scales, const float* __restrict__ means,
                     const float* __restrict__ noise, float* __restrict__ xt_out, float* __restrict__ lik, int total,
                     float scale_bound) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float mu = means ? means[i] : 0.0f;
  const float xv = x[i];
  const float xt = noise ? xv + noise[i] : (means ? rintf(xv - mu) + mu : rintf(xv));
  const float s = fmaxf(scales[i], scale_bound);
  const float val = fabsf(means ? xt - mu : xt);
  const float c = -0.70710678118654752440f;
  const float up = 0.5f * erfcf(c * ((0.5f - val) / s));
  const float lo = 0.5f * erfcf(c * ((-0.5f - val) / s));
  lik[i] = fmaxf(up - lo, 1e-9f);
  if (xt_out) xt_out[i] = xt;
}

extern "C" int tmae_gc_likelihood_fwd(const float* x, const float* scales, const float* means, const float* noise,
                                      float* x_tilde, float* lik, int total, float scale_bound, void* stream) {
  if (total <= 0) return TMAE_OK;
  hipLaunchKernelGGL(gc_likelihood_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x, scales,
                     means, noise, x_tilde, lik, total, scale_bound);
  TMAE_LAUNCH_CHECK("tmae_gc_likelihood_fwd");
}

// ------------------------------------------------------------------ entropy-coding support (MCM.compress / decompress)
// EntropyBottleneck.update (compressai; called through CompressionModel.update, testing.py:223):
// pmf[c][j] = |sigmoid(s f(x + 1/2)) - sigmoid(s f(x - 1/2))| at x = pmf_start[c] + j, s = -sign(lower + upper),
// tail[c] = sigmoid(lower[c][0]) + sigmoid(-upper[c][max_length - 1])  (upstream uses the LAST sample of the
// padded range for every channel, not of the channel's own length; restated as is).
__global__ void __launch_bounds__(256)
eb_pmf_kernel(const float* __restrict__ tab, const float* __restrict__ pmf_start, int C, int max_length,
              float* __restrict__ pmf, float* __restrict__ tail) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= C * max_length) return;
  const int c = i / max_length, j = i - c * max_length;
  const float* t = tab + (size_t)c * EB_PACK;
  const float x = (float)j + pmf_start[c];
  const float lower = eb_logits(t, x - 0.5f);
  const float upper = eb_logits(t, x + 0.5f);
  const float sum = lower + upper;
  const float sgn = sum > 0.0f ? -1.0f : (sum < 0.0f ? 1.0f : -0.0f);
  pmf[i] = fabsf(sigmoid_t(sgn * upper) - sigmoid_t(sgn * lower));
  if (j == 0) {
    const float xl = (float)(max_length - 1) + pmf_start[c];
    tail[c] = sigmoid_t(lower) + sigmoid_t(-eb_logits(t, xl + 0.5f));
  }
}

extern "C" int tmae_eb_pmf(const tmae_eb_params* params, float* table, const float* pmf_start, int C, int max_length,
                           float* pmf, float* tail, void* stream) {
  TMAE_REQUIRE(params && table && pmf_start && pmf && tail && C > 0 && max_length > 0, "tmae_eb_pmf: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(eb_prep_kernel, dim3(ceil_div(C * EB_PACK, 256)), dim3(256), 0, st, *params, table, C);
  hipLaunchKernelGGL(eb_pmf_kernel, dim3(ceil_div(C * max_length, 256)), dim3(256), 0, st, table, pmf_start, C,
                     max_length, pmf, tail);
  TMAE_LAUNCH_CHECK("tmae_eb_pmf");
}

// EntropyBottleneck.compress: symbols = round(z - median) (quantize "symbols"); z NHWC [n*HW][C],
// symbols NCHW [n][C][HW] (compressai codes symbols[i].reshape(-1) per image, channel-major)
__global__ void __launch_bounds__(256)
eb_symbols_kernel(const float* __restrict__ z, const float* __restrict__ tab, int C, int HW, int total,
                  int* __restrict__ sym) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C, m = i / C;
  const int b = m / HW, pix = m - b * HW;
  sym[((size_t)b * C + c) * HW + pix] = (int)rintf(z[i] - tab[(size_t)c * EB_PACK + 58]);
}

// EntropyBottleneck.decompress: z_hat = symbols + median (dequantize), symbols NCHW -> z_hat NHWC
__global__ void __launch_bounds__(256)
eb_dequantize_kernel(const int* __restrict__ sym, const float* __restrict__ tab, int C, int HW, int total,
                     void* __restrict__ zhat, int zhat_bf16) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = i % C, m = i / C;
  const int b = m / HW, pix = m - b * HW;
  const float v = (float)sym[((size_t)b * C + c) * HW + pix] + tab[(size_t)c * EB_PACK + 58];
  if (zhat_bf16) ((bf16*)zhat)[i] = (bf16)v;
  else ((float*)zhat)[i] = v;
}

extern "C" int tmae_eb_symbols(const float* z, const tmae_eb_params* params, float* table, int n, int C, int HW,
                               int* symbols, void* stream) {
  TMAE_REQUIRE(z && params && table && symbols, "tmae_eb_symbols: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(eb_prep_kernel, dim3(ceil_div(C * EB_PACK, 256)), dim3(256), 0, st, *params, table, C);
  const int total = n * HW * C;
  if (total > 0)
    hipLaunchKernelGGL(eb_symbols_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, z, table, C, HW, total,
                       symbols);
  TMAE_LAUNCH_CHECK("tmae_eb_symbols");
}

extern "C" int tmae_eb_dequantize(const int* symbols, const tmae_eb_params* params, float* table, int n, int C, int HW,
                                  void* zhat, int zhat_dtype, void* stream) {
  TMAE_REQUIRE(symbols && params && table && zhat, "tmae_eb_dequantize: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(eb_prep_kernel, dim3(ceil_div(C * EB_PACK, 256)), dim3(256), 0, st, *params, table, C);
  const int total = n * HW * C;
  if (total > 0)
    hipLaunchKernelGGL(eb_dequantize_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, st, symbols, table, C, HW,
                       total, zhat, zhat_dtype == TMAE_BF16);
  TMAE_LAUNCH_CHECK("tmae_eb_dequantize");
}
