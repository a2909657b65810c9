// Distortion terms of MCM.forward_loss (reference MCM.py:690-712): SSIM (pytorch_msssim semantics:
// 11-tap gaussian window, sigma 1.5, "valid" separable filtering, K = (0.01, 0.03), data range 1,
// mean over every channel map) and L1, forward and backward, over NCHW f32 planes.
//
// forward:  hpass  (x, y, x^2, y^2, xy filtered along W)           -> 5 maps [P][H][Wo]
//           vpass  (filtered along H; per output pixel S and dS/d{mu_x, E[x^2], E[xy]}) -> 3 maps [P][Ho][Wo]
//                  + fixed-grid f64 partial sums of S and |x - y|
// backward: the transposed filters of the 3 derivative maps (H then W), combined with x and y:
//           dL/dx = -g_ssim / N_out * (G^T D1 + 2 x G^T D2 + y G^T D3) + g_l1 * sign(x - y) / N_in
#include "common.h"

#define SS_WIN 11
#define SS_BLOCKS 1024

struct SsimWin { float g[SS_WIN]; };

static SsimWin ssim_window(float sigma) {
  SsimWin w;
  double s = 0.0, v[SS_WIN];
  for (int i = 0; i < SS_WIN; ++i) {
    const double c = (double)(i - SS_WIN / 2);
    v[i] = exp(-(c * c) / (2.0 * (double)sigma * sigma));
    s += v[i];
  }
  for (int i = 0; i < SS_WIN; ++i) w.g[i] = (float)(v[i] / s);
  return w;
}

__global__ void __launch_bounds__(256)
ssim_hpass_kernel(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ h, int P, int H, int W,
                  SsimWin win) {
  const int Wo = W - (SS_WIN - 1);
  const long long plane = (long long)H * Wo;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)P * plane) return;
  const int p = (int)(i / plane);
  const int rem = (int)(i - (long long)p * plane);
  const int r = rem / Wo, c = rem - r * Wo;
  const float* xr = x + ((size_t)p * H + r) * W + c;
  const float* yr = y + ((size_t)p * H + r) * W + c;
  float a = 0.f, b = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
  for (int t = 0; t < SS_WIN; ++t) {
    const float xv = xr[t], yv = yr[t], g = win.g[t];
    a += g * xv;
    b += g * yv;
    aa += g * xv * xv;
    bb += g * yv * yv;
    ab += g * xv * yv;
  }
  const long long n = (long long)P * plane;
  h[i] = a;
  h[n + i] = b;
  h[2 * n + i] = aa;
  h[3 * n + i] = bb;
  h[4 * n + i] = ab;
}

__global__ void __launch_bounds__(256)
ssim_vpass_kernel(const float* __restrict__ h, float* __restrict__ d, int P, int H, int W, SsimWin win, float c1,
                  float c2, double* __restrict__ part, long long total) {
  __shared__ double red[256];
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long hplane = (long long)H * Wo, oplane = (long long)Ho * Wo;
  const long long nh = (long long)P * hplane, no = (long long)P * oplane;
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int p = (int)(i / oplane);
    const int rem = (int)(i - (long long)p * oplane);
    const int r = rem / Wo, c = rem - r * Wo;
    const float* hb = h + (size_t)p * hplane + (size_t)r * Wo + c;
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
    for (int t = 0; t < SS_WIN; ++t) {
      const float g = win.g[t];
      const size_t o = (size_t)t * Wo;
      m1 += g * hb[o];
      m2 += g * hb[nh + o];
      e11 += g * hb[2 * nh + o];
      e22 += g * hb[3 * nh + o];
      e12 += g * hb[4 * nh + o];
    }
    const float s11 = e11 - m1 * m1, s22 = e22 - m2 * m2, s12 = e12 - m1 * m2;
    const float A1 = 2.f * m1 * m2 + c1, B1 = m1 * m1 + m2 * m2 + c1;
    const float A2 = 2.f * s12 + c2, B2 = s11 + s22 + c2;
    const float l = A1 / B1, cs = A2 / B2;
    acc += (double)(l * cs);
    if (d) {
      const float dl = (2.f * m2 * B1 - A1 * 2.f * m1) / (B1 * B1);
      const float dcs = (-2.f * m2 * B2 + A2 * 2.f * m1) / (B2 * B2);
      d[i] = dl * cs + l * dcs;             // dS / d mu_x
      d[no + i] = -l * A2 / (B2 * B2);      // dS / d E[x^2]
      d[2 * no + i] = l * 2.f / B2;         // dS / d E[xy]
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256)
l1_partial_kernel(const float* __restrict__ x, const float* __restrict__ y, long long n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    s += (double)fabsf(x[i] - y[i]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// out[0] = 1 - mean S, out[1] = mean |x - y|
__global__ void __launch_bounds__(256)
distortion_final_kernel(const double* __restrict__ ps, const double* __restrict__ pl, int np, double n_out, double n_in,
                        float* __restrict__ out) {
  __shared__ double r1[256], r2[256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) {
    a += ps[i];
    b += pl[i];
  }
  r1[threadIdx.x] = a;
  r2[threadIdx.x] = b;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      r1[threadIdx.x] += r1[threadIdx.x + o];
      r2[threadIdx.x] += r2[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = (float)(1.0 - r1[0] / n_out);
    out[1] = (float)(r2[0] / n_in);
  }
}

extern "C" int tmae_distortion_fwd(const float* x, const float* y, int P, int H, int W, float* hwork, float* dmaps,
                                   double* part, float* out, void* stream) {
  TMAE_REQUIRE(x && y && hwork && part && out && H >= SS_WIN && W >= SS_WIN, "tmae_distortion_fwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const SsimWin win = ssim_window(1.5f);
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long nh = (long long)P * H * Wo, no = (long long)P * Ho * Wo, ni = (long long)P * H * W;
  hipLaunchKernelGGL(ssim_hpass_kernel, dim3((unsigned)((nh + 255) / 256)), dim3(256), 0, st, x, y, hwork, P, H, W, win);
  hipLaunchKernelGGL(ssim_vpass_kernel, dim3(SS_BLOCKS), dim3(256), 0, st, hwork, dmaps, P, H, W, win, 0.01f * 0.01f,
                     0.03f * 0.03f, part, no);
  hipLaunchKernelGGL(l1_partial_kernel, dim3(SS_BLOCKS), dim3(256), 0, st, x, y, ni, part + SS_BLOCKS);
  hipLaunchKernelGGL(distortion_final_kernel, dim3(1), dim3(256), 0, st, part, part + SS_BLOCKS, SS_BLOCKS, (double)no,
                     (double)ni, out);
  TMAE_LAUNCH_CHECK("tmae_distortion_fwd");
}

// transposed vertical filter of the 3 derivative maps: v[k][p][r][c] = sum_t g[t] d[k][p][r - t][c], r in [0, H)
__global__ void __launch_bounds__(256)
ssim_bwd_vpass_kernel(const float* __restrict__ d, float* __restrict__ v, int P, int H, int W, SsimWin win) {
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long vplane = (long long)H * Wo, oplane = (long long)Ho * Wo;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)P * vplane) return;
  const int p = (int)(i / vplane);
  const int rem = (int)(i - (long long)p * vplane);
  const int r = rem / Wo, c = rem - r * Wo;
  const long long no = (long long)P * oplane, nv = (long long)P * vplane;
  float a = 0.f, b = 0.f, e = 0.f;
#pragma unroll
  for (int t = 0; t < SS_WIN; ++t) {
    const int rr = r - t;
    if (rr >= 0 && rr < Ho) {
      const size_t o = (size_t)p * oplane + (size_t)rr * Wo + c;
      const float g = win.g[t];
      a += g * d[o];
      b += g * d[no + o];
      e += g * d[2 * no + o];
    }
  }
  v[i] = a;
  v[nv + i] = b;
  v[2 * nv + i] = e;
}

__global__ void __launch_bounds__(256)
ssim_bwd_hpass_kernel(const float* __restrict__ v, const float* __restrict__ x, const float* __restrict__ y,
                      float* __restrict__ gx, int P, int H, int W, SsimWin win, const float* __restrict__ gout,
                      float inv_out, float inv_in) {
  const int Wo = W - (SS_WIN - 1);
  const long long iplane = (long long)H * W, vplane = (long long)H * Wo;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)P * iplane) return;
  const int p = (int)(i / iplane);
  const int rem = (int)(i - (long long)p * iplane);
  const int r = rem / W, c = rem - r * W;
  const long long nv = (long long)P * vplane;
  float a = 0.f, b = 0.f, e = 0.f;
#pragma unroll
  for (int t = 0; t < SS_WIN; ++t) {
    const int cc = c - t;
    if (cc >= 0 && cc < Wo) {
      const size_t o = (size_t)p * vplane + (size_t)r * Wo + cc;
      const float g = win.g[t];
      a += g * v[o];
      b += g * v[nv + o];
      e += g * v[2 * nv + o];
    }
  }
  const float xv = x[i], yv = y[i];
  const float gs = gout ? gout[0] : 0.0f, gl = gout ? gout[1] : 0.0f;
  const float diff = xv - yv;
  const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
  gx[i] = -gs * inv_out * (a + 2.f * xv * b + yv * e) + gl * inv_in * sg;
}

extern "C" int tmae_distortion_bwd(const float* x, const float* y, int P, int H, int W, const float* dmaps, float* vwork,
                                   const float* gout, float* gx, void* stream) {
  TMAE_REQUIRE(x && y && dmaps && vwork && gout && gx, "tmae_distortion_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const SsimWin win = ssim_window(1.5f);
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long nv = (long long)P * H * Wo, ni = (long long)P * H * W;
  hipLaunchKernelGGL(ssim_bwd_vpass_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, st, dmaps, vwork, P, H, W,
                     win);
  hipLaunchKernelGGL(ssim_bwd_hpass_kernel, dim3((unsigned)((ni + 255) / 256)), dim3(256), 0, st, vwork, x, y, gx, P, H,
                     W, win, gout, (float)(1.0 / ((double)P * Ho * Wo)), (float)(1.0 / (double)ni));
  TMAE_LAUNCH_CHECK("tmae_distortion_bwd");
}
