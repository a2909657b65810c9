// Distortion terms of MCM.forward_loss (reference MCM.py:690-712): SSIM (pytorch_msssim semantics:
// 11-tap gaussian window, sigma 1.5, "valid" separable filtering, K = (0.01, 0.03), data range 1,
// mean over every channel map) and L1, forward and backward, over NCHW f32 planes.
//
// forward:  per 32 x 64 output tile, x and y through LDS: filtered along W (x, y, x^2, y^2, xy), then along H;
//           per output pixel S and dS/d{mu_x, E[x^2], E[xy]} -> 3 maps [P][Ho][Wo]; f64 partial sums of S per
//           tile and of |x - y| over a fixed grid
// backward: per 32 x 64 input tile, the transposed filters of the 3 derivative maps (H then W) through LDS,
//           combined with x and y:
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

// ---- forward, one workgroup per (plane, 32 x 64 output tile): the (32 + 10) x (64 + 10) x / y patch goes to LDS,
// the horizontal pass writes the 5 filtered maps of its 42 rows to LDS, the vertical pass forms S and the three
// derivative maps per output pixel.  Per-pixel arithmetic is the separable filter in tap order (h then v);
// S is summed per workgroup in f64 into one partial per tile (fixed grid, folded in index order).
#define SS_TH 32
#define SS_TW 64
#ifndef SS_NT
#define SS_NT 512  // threads per tile workgroup: 8 waves, two workgroups (78.6 / 65.7 KB of LDS) per CU
#endif
#define SS_IH (SS_TH + SS_WIN - 1)
#define SS_IW (SS_TW + SS_WIN - 1)
#define SS_VR 4  // output rows per vertical-pass item (register blocking of the filtered rows)
#define SS_IWP 76  // x / y patch row pitch: 74 columns padded to whole 16-B chunks (the h pass reads 4 at a time)

__global__ void __launch_bounds__(SS_NT)
ssim_fwd_tile_kernel(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ d, int P, int H,
                     int W, SsimWin win, float c1, float c2, double* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float xs[SS_IH][SS_IWP], ys[SS_IH][SS_IWP];
  __shared__ __attribute__((aligned(16))) float hm[5][SS_IH][SS_TW];
  __shared__ double red[SS_NT / 64];
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const int tx = (Wo + SS_TW - 1) / SS_TW, ty = (Ho + SS_TH - 1) / SS_TH;
  const int t = threadIdx.x;
  int b = blockIdx.x;
  const int p = b / (tx * ty);
  b -= p * tx * ty;
  const int r0 = (b / tx) * SS_TH, c0 = (b % tx) * SS_TW;
  const float* xp = x + (size_t)p * H * W;
  const float* yp = y + (size_t)p * H * W;
  for (int e = t; e < SS_IH * SS_IWP; e += SS_NT) {
    const int rr = e / SS_IWP, cc = e - rr * SS_IWP;
    const int r = r0 + rr, c = c0 + cc;
    const bool in = cc < SS_IW && r < H && c < W;
    xs[rr][cc] = in ? xp[(size_t)r * W + c] : 0.0f;
    ys[rr][cc] = in ? yp[(size_t)r * W + c] : 0.0f;
  }
  __syncthreads();
  // horizontal pass: one item = one row x 4 consecutive columns, its 14 x and y values read as 16-B LDS loads
  for (int e = t; e < SS_IH * (SS_TW / 4); e += SS_NT) {
    const int rr = e / (SS_TW / 4), cc = 4 * (e - rr * (SS_TW / 4));
    float xv[16], yv[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4 a4 = *reinterpret_cast<const f32x4*>(&xs[rr][cc + 4 * q]);
      const f32x4 b4 = *reinterpret_cast<const f32x4*>(&ys[rr][cc + 4 * q]);
#pragma unroll
      for (int j = 0; j < 4; ++j) { xv[4 * q + j] = a4[j]; yv[4 * q + j] = b4[j]; }
    }
    f32x4 o0, o1, o2, o3, o4;
#pragma unroll
    for (int o = 0; o < 4; ++o) {
      float a = 0.f, bb_ = 0.f, aa = 0.f, bb = 0.f, ab = 0.f;
#pragma unroll
      for (int k = 0; k < SS_WIN; ++k) {
        const float xk = xv[o + k], yk = yv[o + k], g = win.g[k];
        a += g * xk;
        bb_ += g * yk;
        aa += g * xk * xk;
        bb += g * yk * yk;
        ab += g * xk * yk;
      }
      o0[o] = a; o1[o] = bb_; o2[o] = aa; o3[o] = bb; o4[o] = ab;
    }
    *reinterpret_cast<f32x4*>(&hm[0][rr][cc]) = o0;
    *reinterpret_cast<f32x4*>(&hm[1][rr][cc]) = o1;
    *reinterpret_cast<f32x4*>(&hm[2][rr][cc]) = o2;
    *reinterpret_cast<f32x4*>(&hm[3][rr][cc]) = o3;
    *reinterpret_cast<f32x4*>(&hm[4][rr][cc]) = o4;
  }
  __syncthreads();
  const long long no = (long long)P * Ho * Wo;
  double acc = 0.0;
  // each item: one column, SS_VR consecutive output rows; the SS_VR + 10 filtered rows it needs are read from LDS
  // once (per output the taps still accumulate in order 0..10, as one output per item would)
  for (int e = t; e < (SS_TH / SS_VR) * SS_TW; e += SS_NT) {
    const int rs = e / SS_TW, cc = e - rs * SS_TW;
    const int rr0 = rs * SS_VR;
    float hv[5][SS_VR + SS_WIN - 1];
#pragma unroll
    for (int m = 0; m < 5; ++m)
#pragma unroll
      for (int k = 0; k < SS_VR + SS_WIN - 1; ++k) hv[m][k] = hm[m][rr0 + k][cc];
#pragma unroll
    for (int o = 0; o < SS_VR; ++o) {
      const int r = r0 + rr0 + o, c = c0 + cc;
      if (r >= Ho || c >= Wo) continue;
      float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
#pragma unroll
      for (int k = 0; k < SS_WIN; ++k) {
        const float g = win.g[k];
        m1 += g * hv[0][o + k];
        m2 += g * hv[1][o + k];
        e11 += g * hv[2][o + k];
        e22 += g * hv[3][o + k];
        e12 += g * hv[4][o + k];
      }
      const float s11 = e11 - m1 * m1, s22 = e22 - m2 * m2, s12 = e12 - m1 * m2;
      const float A1 = 2.f * m1 * m2 + c1, B1 = m1 * m1 + m2 * m2 + c1;
      const float A2 = 2.f * s12 + c2, B2 = s11 + s22 + c2;
      const float l = A1 / B1, cs = A2 / B2;
      acc += (double)(l * cs);
      if (d) {
        const long long i = ((long long)p * Ho + r) * Wo + c;
        const float dl = (2.f * m2 * B1 - A1 * 2.f * m1) / (B1 * B1);
        const float dcs = (-2.f * m2 * B2 + A2 * 2.f * m1) / (B2 * B2);
        d[i] = dl * cs + l * dcs;             // dS / d mu_x
        d[no + i] = -l * A2 / (B2 * B2);      // dS / d E[x^2]
        d[2 * no + i] = l * 2.f / B2;         // dS / d E[xy]
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((t & 63) == 0) red[t >> 6] = acc;
  __syncthreads();
  if (t == 0) {
    double sum = 0.0;
#pragma unroll
    for (int w = 0; w < SS_NT / 64; ++w) sum += red[w];
    part[blockIdx.x] = sum;
  }
}

__global__ void __launch_bounds__(256)
l1_partial_kernel(const float* __restrict__ x, const float* __restrict__ y, long long n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const long long n4 = ((((size_t)x | (size_t)y) & 15) == 0) ? n / 4 : 0;  // 16-B loads over the aligned body
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(x + 4 * i), b = *reinterpret_cast<const f32x4*>(y + 4 * i);
    s += (double)(fabsf(a[0] - b[0]) + fabsf(a[1] - b[1])) + (double)(fabsf(a[2] - b[2]) + fabsf(a[3] - b[3]));
  }
  for (long long i = 4 * n4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
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
distortion_final_kernel(const double* __restrict__ ps, int nps, const double* __restrict__ pl, int npl, double n_out,
                        double n_in, float* __restrict__ out) {
  __shared__ double r1[256], r2[256];
  double a = 0.0, b = 0.0;
  for (int i = threadIdx.x; i < nps; i += 256) a += ps[i];
  for (int i = threadIdx.x; i < npl; i += 256) b += pl[i];
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

static inline int ssim_tiles(int P, int Ho, int Wo) {
  return P * ((Ho + SS_TH - 1) / SS_TH) * ((Wo + SS_TW - 1) / SS_TW);
}

extern "C" int tmae_distortion_fwd(const float* x, const float* y, int P, int H, int W, float* hwork, float* dmaps,
                                   double* part, float* out, void* stream) {
  TMAE_REQUIRE(x && y && hwork && part && out && H >= SS_WIN && W >= SS_WIN, "tmae_distortion_fwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const SsimWin win = ssim_window(1.5f);
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long no = (long long)P * Ho * Wo, ni = (long long)P * H * W;
  TMAE_REQUIRE(no < (1ll << 31) && ni < (1ll << 31), "tmae_distortion_fwd: %lld pixels exceed the 32-bit index range",
               ni);
  // one f64 partial per tile, kept in the caller's hwork (>= 5 P H (W - 10) floats, far more than the tiles)
  const int nt = ssim_tiles(P, Ho, Wo);
  TMAE_REQUIRE(2ll * nt <= 5ll * P * H * Wo, "tmae_distortion_fwd: workspace");
  double* tpart = reinterpret_cast<double*>(hwork);
  hipLaunchKernelGGL(ssim_fwd_tile_kernel, dim3((unsigned)nt), dim3(SS_NT), 0, st, x, y, dmaps, P, H, W, win,
                     0.01f * 0.01f, 0.03f * 0.03f, tpart);
  hipLaunchKernelGGL(l1_partial_kernel, dim3(SS_BLOCKS), dim3(256), 0, st, x, y, ni, part + SS_BLOCKS);
  hipLaunchKernelGGL(distortion_final_kernel, dim3(1), dim3(256), 0, st, tpart, nt, part + SS_BLOCKS, SS_BLOCKS,
                     (double)no, (double)ni, out);
  TMAE_LAUNCH_CHECK("tmae_distortion_fwd");
}

// ---- backward, one workgroup per (plane, 32 x 64 INPUT tile): the three derivative maps over the rows and
// columns the tile's transposed filters reach ((32 + 10) x (64 + 10), zero outside the valid output) go to LDS;
// the transposed vertical filter v[k][r][c'] = sum_t g[t] d[k][r - t][c'] for the tile's rows and columns
// c0 - 10 .. c0 + 63 to LDS; then gx[r][c] = -g_ssim / N_out (G^T D1 + 2 x G^T D2 + y G^T D3) + g_l1 sign(x - y) / N_in
// with the transposed horizontal filter.  Taps outside the valid output add g * 0.
__global__ void __launch_bounds__(SS_NT)
ssim_bwd_tile_kernel(const float* __restrict__ d, const float* __restrict__ x, const float* __restrict__ y,
                     float* __restrict__ gx, int P, int H, int W, SsimWin win, const float* __restrict__ gout,
                     float inv_out, float inv_in) {
  __shared__ float ds[3][SS_IH][SS_IW];
  __shared__ __attribute__((aligned(16))) float vs[3][SS_TH][SS_IWP];
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const int tx = (W + SS_TW - 1) / SS_TW, ty = (H + SS_TH - 1) / SS_TH;
  const int t = threadIdx.x;
  int b = blockIdx.x;
  const int p = b / (tx * ty);
  b -= p * tx * ty;
  const int r0 = (b / tx) * SS_TH, c0 = (b % tx) * SS_TW;
  const long long no = (long long)P * Ho * Wo;
  const float* dp = d + (size_t)p * Ho * Wo;
  // ds[k][i][j] = d[k][r0 - 10 + i][c0 - 10 + j]
  for (int e = t; e < SS_IH * SS_IW; e += SS_NT) {
    const int i = e / SS_IW, j = e - i * SS_IW;
    const int r = r0 - (SS_WIN - 1) + i, c = c0 - (SS_WIN - 1) + j;
    const bool in = r >= 0 && r < Ho && c >= 0 && c < Wo;
    const size_t o = (size_t)r * Wo + c;
#pragma unroll
    for (int k = 0; k < 3; ++k) ds[k][i][j] = in ? dp[k * no + o] : 0.0f;
  }
  __syncthreads();
  // vs[k][i][j] = v[k][r0 + i][c0 - 10 + j] = sum_t g[t] d[k][r0 + i - t][...] = sum_t g[t] ds[k][i + 10 - t][j]
  for (int e = t; e < (SS_TH / SS_VR) * SS_IW; e += SS_NT) {  // SS_VR rows per item, as in the forward
    const int is = e / SS_IW, j = e - is * SS_IW;
    const int i0 = is * SS_VR;
    float dv[3][SS_VR + SS_WIN - 1];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int k = 0; k < SS_VR + SS_WIN - 1; ++k) dv[m][k] = ds[m][i0 + k][j];
#pragma unroll
    for (int o = 0; o < SS_VR; ++o) {
      float a = 0.f, bq = 0.f, q = 0.f;
#pragma unroll
      for (int k = 0; k < SS_WIN; ++k) {
        const float g = win.g[k];
        a += g * dv[0][o + SS_WIN - 1 - k];
        bq += g * dv[1][o + SS_WIN - 1 - k];
        q += g * dv[2][o + SS_WIN - 1 - k];
      }
      vs[0][i0 + o][j] = a;
      vs[1][i0 + o][j] = bq;
      vs[2][i0 + o][j] = q;
    }
  }
  __syncthreads();
  const float gs = gout ? gout[0] : 0.0f, gl = gout ? gout[1] : 0.0f;
  const bool aligned16 = (((size_t)x | (size_t)y | (size_t)gx) & 15) == 0;
  // transposed horizontal pass + the combination with x and y: one item = one row x 4 consecutive columns, the
  // 14 v values of each map read as 16-B LDS loads, x / y / dx as 16-B global accesses
  for (int e = t; e < SS_TH * (SS_TW / 4); e += SS_NT) {
    const int i = e / (SS_TW / 4), j = 4 * (e - i * (SS_TW / 4));
    const int r = r0 + i, c = c0 + j;
    if (r >= H || c >= W) continue;
    float vv[3][16];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const f32x4 v4 = *reinterpret_cast<const f32x4*>(&vs[m][i][j + 4 * q4]);
#pragma unroll
        for (int u = 0; u < 4; ++u) vv[m][4 * q4 + u] = v4[u];
      }
    const size_t o = ((size_t)p * H + r) * W + c;
    // 16-B accesses only on 16-B aligned bases: an offset view (a sliced batch) takes the per-element path
    const bool full = c + 4 <= W && (W & 3) == 0 && aligned16;
    f32x4 xv4, yv4, gv4;
    if (full) {
      xv4 = *reinterpret_cast<const f32x4*>(x + o);
      yv4 = *reinterpret_cast<const f32x4*>(y + o);
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        xv4[u] = c + u < W ? x[o + u] : 0.f;
        yv4[u] = c + u < W ? y[o + u] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float a = 0.f, bq = 0.f, q = 0.f;
#pragma unroll
      for (int k = 0; k < SS_WIN; ++k) {  // v column c + u - k = vs column j + u + 10 - k
        const float g = win.g[k];
        a += g * vv[0][u + SS_WIN - 1 - k];
        bq += g * vv[1][u + SS_WIN - 1 - k];
        q += g * vv[2][u + SS_WIN - 1 - k];
      }
      const float xv = xv4[u], yv = yv4[u];
      const float diff = xv - yv;
      const float sg = diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f);
      gv4[u] = -gs * inv_out * (a + 2.f * xv * bq + yv * q) + gl * inv_in * sg;
    }
    if (full) {
      *reinterpret_cast<f32x4*>(gx + o) = gv4;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (c + u < W) gx[o + u] = gv4[u];
    }
  }
}

extern "C" int tmae_distortion_bwd(const float* x, const float* y, int P, int H, int W, const float* dmaps, float* vwork,
                                   const float* gout, float* gx, void* stream) {
  TMAE_REQUIRE(x && y && dmaps && gout && gx && H >= SS_WIN && W >= SS_WIN, "tmae_distortion_bwd: bad arguments");
  (void)vwork;  // the transposed vertical pass lives in LDS since round 4
  hipStream_t st = (hipStream_t)stream;
  const SsimWin win = ssim_window(1.5f);
  const int Wo = W - (SS_WIN - 1), Ho = H - (SS_WIN - 1);
  const long long ni = (long long)P * H * W;
  TMAE_REQUIRE(ni < (1ll << 31), "tmae_distortion_bwd: %lld pixels exceed the 32-bit index range", ni);
  const int nt = P * ((H + SS_TH - 1) / SS_TH) * ((W + SS_TW - 1) / SS_TW);
  hipLaunchKernelGGL(ssim_bwd_tile_kernel, dim3((unsigned)nt), dim3(SS_NT), 0, st, dmaps, x, y, gx, P, H, W, win, gout,
                     (float)(1.0 / ((double)P * Ho * Wo)), (float)(1.0 / (double)ni));
  TMAE_LAUNCH_CHECK("tmae_distortion_bwd");
}
