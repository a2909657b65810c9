// LayerNorm over the fp32 residual stream (timm Block norm1/norm2, MCM encoder_norm /
// decoder_norm; eps = 1e-6 from MCM.py:46).  One wave per row, 16-B vector loads, two-pass
// mean/variance in registers, output cast to the GEMM operand type.  A row remap lets the same
// kernel drop cls rows (MCM.py:631-632, 680-686) without a copy:
//   source row = (r / G) * Gs + off + (r % G)
#include "common.h"

template <typename OT, int VPL>
__global__ void __launch_bounds__(256)
layernorm_kernel(const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
                 OT* __restrict__ y, int rows, int D, int G, int Gs, int off, float eps) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int sr = (r / G) * Gs + off + (r % G);
  const float* xr = x + (size_t)sr * D;
  const int nch = D >> 2;
  // gamma / beta are loaded with the row, so the wave's only dependent memory latency is the row itself
  f32x4 v[VPL], gv[VPL], bv[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    v[i] = (c < nch) ? load4f(xr + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    gv[i] = (c < nch) ? load4f(gamma + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    bv[i] = (c < nch) ? load4f(beta + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  const float mean = s / (float)D;
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[i][j] - mean;
        q += d * d;
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  const float rstd = 1.0f / sqrtf(q / (float)D + eps);
  OT* yr = y + (size_t)r * D;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (v[i][j] - mean) * rstd * gv[i][j] + bv[i][j];
      store4(yr + 4 * c, o);
    }
  }
}

template <typename OT>
static int ln_launch(const float* x, const float* g, const float* b, void* y, int rows, int D, int G, int Gs, int off,
                     float eps, hipStream_t st) {
  const int grid = ceil_div(rows, 4);
  if (rows == 0) return TMAE_OK;
  const int vpl = ceil_div(D / 4, 64);
#define TMAE_LN(V) hipLaunchKernelGGL((layernorm_kernel<OT, V>), dim3(grid), dim3(256), 0, st, x, g, b, (OT*)y, rows, D, G, Gs, off, eps)
  if (vpl <= 1) TMAE_LN(1);
  else if (vpl <= 2) TMAE_LN(2);
  else if (vpl <= 3) TMAE_LN(3);
  else if (vpl <= 4) TMAE_LN(4);
  else TMAE_LN(8);
#undef TMAE_LN
  TMAE_LAUNCH_CHECK("tmae_layernorm_fwd");
}

extern "C" int tmae_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, int rows, int D,
                                  int row_group, int group_stride, int row_offset, float eps, int out_dtype,
                                  void* stream) {
  TMAE_REQUIRE(D % 4 == 0 && D <= 2048, "tmae_layernorm_fwd: D=%d must be a multiple of 4 and <= 2048", D);
  TMAE_REQUIRE(row_group > 0, "tmae_layernorm_fwd: row_group must be > 0");
  if (out_dtype == TMAE_BF16)
    return ln_launch<bf16>(x, gamma, beta, y, rows, D, row_group, group_stride, row_offset, eps, (hipStream_t)stream);
  return ln_launch<float>(x, gamma, beta, y, rows, D, row_group, group_stride, row_offset, eps, (hipStream_t)stream);
}
