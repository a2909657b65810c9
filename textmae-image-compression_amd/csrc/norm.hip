// LayerNorm over the fp32 residual stream (timm Block norm1/norm2, MCM encoder_norm /
// decoder_norm; eps = 1e-6 from MCM.py:46).  One wave per row, 16-B vector loads, two-pass
// mean/variance in registers, output cast to the GEMM operand type.  A row remap lets the same
// kernel drop cls rows (MCM.py:631-632, 680-686) without a copy:
//   source row = (r / G) * Gs + off + (r % G)
#include "common.h"

// RPW rows per wave: gamma / beta loaded once per wave, all RPW rows' loads in flight together.  Measured
// slower at the bench shapes (42 launches: 390 us at 4 or 2 rows per wave, 348 us at 1 -- fewer waves hide
// less latency), so the launcher instantiates one row per wave only.
template <typename OT, int VPL, int RPW>
__global__ void __launch_bounds__(256)
layernorm_kernel(const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
                 OT* __restrict__ y, int rows, int D, int G, int Gs, int off, float eps) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW;
  if (r0 >= rows) return;
  const int nch = D >> 2;
  f32x4 v[RPW][VPL], gv[VPL], bv[VPL];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int r = r0 + k;
    const float* xr = x + (size_t)((r / G) * Gs + off + (r % G)) * D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      v[k][i] = (c < nch && r < rows) ? load4f(xr + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    gv[i] = (c < nch) ? load4f(gamma + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    bv[i] = (c < nch) ? load4f(beta + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float s[RPW], q[RPW];
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    s[k] = 0.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) s[k] += (v[k][i][0] + v[k][i][1]) + (v[k][i][2] + v[k][i][3]);
  }
#ifdef TMAE_LN_SHFL  // A/B builds: the ds_bpermute butterfly
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < RPW; ++k) s[k] += __shfl_xor(s[k], o);
#else
#pragma unroll
  for (int k = 0; k < RPW; ++k) s[k] = wave_allsum(s[k]);
#endif
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const float mean = s[k] / (float)D;
    s[k] = mean;
    q[k] = 0.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[k][i][j] - mean;
          q[k] += d * d;
        }
      }
    }
  }
#ifdef TMAE_LN_SHFL
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int k = 0; k < RPW; ++k) q[k] += __shfl_xor(q[k], o);
#else
#pragma unroll
  for (int k = 0; k < RPW; ++k) q[k] = wave_allsum(q[k]);
#endif
#pragma unroll
  for (int k = 0; k < RPW; ++k) {
    const int r = r0 + k;
    if (r >= rows) break;
    const float mean = s[k];
    const float rstd = 1.0f / sqrtf(q[k] / (float)D + eps);
    OT* yr = y + (size_t)r * D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (v[k][i][j] - mean) * rstd * gv[i][j] + bv[i][j];
        store4(yr + 4 * c, o);
      }
    }
  }
}

template <typename OT>
static int ln_launch(const float* x, const float* g, const float* b, void* y, int rows, int D, int G, int Gs, int off,
                     float eps, hipStream_t st) {
  if (rows == 0) return TMAE_OK;
  const int vpl = ceil_div(D / 4, 64);
  // one row per wave: 2 or 4 rows per wave (gamma / beta loaded once per wave) measured slower (390 vs 348 us per
  // forward, profiles/r02/bench_call40_ln_rpw*.log) -- fewer waves hide less latency
  const int grid = ceil_div(rows, 4);
#define TMAE_LN(V, R) hipLaunchKernelGGL((layernorm_kernel<OT, V, R>), dim3(grid), dim3(256), 0, st, x, g, b, (OT*)y, rows, D, G, Gs, off, eps)
#define TMAE_LN_V(R)            \
  if (vpl <= 1) TMAE_LN(1, R);  \
  else if (vpl <= 2) TMAE_LN(2, R); \
  else if (vpl <= 3) TMAE_LN(3, R); \
  else if (vpl <= 4) TMAE_LN(4, R); \
  else TMAE_LN(8, R);
  TMAE_LN_V(1)
#undef TMAE_LN_V
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
