// Evaluation metrics of the Kodak harness (reference testing.py:40-49, compute_metrics / psnr):
//   org, rec -> round(clamp(255 x, 0, 255)) both; PSNR over the whole batch; MS-SSIM (pytorch_msssim
//   ms_ssim, data_range 255, 11-tap gaussian sigma 1.5, K = (0.01, 0.03), five scales with weights
//   (0.0448, 0.2856, 0.3001, 0.2363, 0.1333), 2x2 average pooling with padding H%2 / W%2 between scales,
//   relu on the per-channel cs / ssim, mean over images and channels).
//
// The work is small (24 Kodak images of 224^2): one workgroup per (image, channel) plane and scale walks
// every output pixel of that plane, f64 partial sums reduced in a fixed order (bitwise reproducible).
// PSNR's squared error is a sum of integers and is kept exact (int64).
#include "common.h"

#define MS_WIN 11
#define MS_LEVELS 5

struct MsWin { float g[MS_WIN]; };

static MsWin ms_window() {
  MsWin w;
  double v[MS_WIN], s = 0.0;
  for (int i = 0; i < MS_WIN; ++i) {
    const double c = (double)(i - MS_WIN / 2);
    v[i] = exp(-(c * c) / (2.0 * 1.5 * 1.5));
    s += v[i];
  }
  for (int i = 0; i < MS_WIN; ++i) w.g[i] = (float)(v[i] / s);
  return w;
}

// q = round(clamp(255 x, 0, 255)) (torch: mul, clamp, round half-to-even)
__global__ void __launch_bounds__(256) quant255_kernel(const float* __restrict__ x, float* __restrict__ q, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) q[i] = rintf(fminf(fmaxf(x[i] * 255.0f, 0.0f), 255.0f));
}

// exact sum of squared differences of two quantised tensors, one partial per block
__global__ void __launch_bounds__(256) sqdiff_kernel(const float* __restrict__ a, const float* __restrict__ b, long long n,
                                                     long long* __restrict__ part) {
  __shared__ long long red[256];
  long long acc = 0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long d = (long long)a[i] - (long long)b[i];
    acc += d * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void psnr_final_kernel(const long long* __restrict__ part, int nparts, long long n, float max_val,
                                  float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  long long s = 0;
  for (int i = 0; i < nparts; ++i) s += part[i];
  const double mse = (double)s / (double)n;
  out[0] = (float)(20.0 * log10((double)max_val) - 10.0 * log10(mse));
}

// per-plane mean of the SSIM map and of the contrast-structure map at one scale ("valid" separable
// gaussian filtering, along H then W as pytorch_msssim's gaussian_filter does)
__global__ void __launch_bounds__(256)
ms_stats_kernel(const float* __restrict__ x, const float* __restrict__ y, int H, int W, MsWin win, float c1, float c2,
                float* __restrict__ ssim_out, float* __restrict__ cs_out) {
  __shared__ double red_s[256], red_c[256];
  const int p = blockIdx.x;
  const bool fh = H >= MS_WIN, fw = W >= MS_WIN;  // pytorch_msssim skips a dimension smaller than the window
  const int th = fh ? MS_WIN : 1, tw = fw ? MS_WIN : 1;
  const int Ho = H - th + 1, Wo = W - tw + 1;
  const float* xp = x + (size_t)p * H * W;
  const float* yp = y + (size_t)p * H * W;
  double as = 0.0, ac = 0.0;
  for (int o = threadIdx.x; o < Ho * Wo; o += 256) {
    const int r = o / Wo, c = o - r * Wo;
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
    for (int j = 0; j < tw; ++j) {
      float h1 = 0.f, h2 = 0.f, h11 = 0.f, h22 = 0.f, h12 = 0.f;
      for (int i = 0; i < th; ++i) {
        const float gi = fh ? win.g[i] : 1.0f;
        const float xv = xp[(size_t)(r + i) * W + c + j], yv = yp[(size_t)(r + i) * W + c + j];
        h1 += gi * xv;
        h2 += gi * yv;
        h11 += gi * (xv * xv);
        h22 += gi * (yv * yv);
        h12 += gi * (xv * yv);
      }
      const float gj = fw ? win.g[j] : 1.0f;
      m1 += gj * h1;
      m2 += gj * h2;
      e11 += gj * h11;
      e22 += gj * h22;
      e12 += gj * h12;
    }
    const float mu11 = m1 * m1, mu22 = m2 * m2, mu12 = m1 * m2;
    const float s11 = e11 - mu11, s22 = e22 - mu22, s12 = e12 - mu12;
    const float cs = (2.0f * s12 + c2) / (s11 + s22 + c2);
    const float ss = ((2.0f * mu12 + c1) / (mu11 + mu22 + c1)) * cs;
    as += (double)ss;
    ac += (double)cs;
  }
  red_s[threadIdx.x] = as;
  red_c[threadIdx.x] = ac;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red_s[threadIdx.x] += red_s[threadIdx.x + s];
      red_c[threadIdx.x] += red_c[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    ssim_out[p] = (float)(red_s[0] / (double)(Ho * Wo));
    cs_out[p] = (float)(red_c[0] / (double)(Ho * Wo));
  }
}

// F.avg_pool2d(kernel 2, stride 2, padding (H % 2, W % 2), count_include_pad=True)
__global__ void __launch_bounds__(256)
avgpool2_kernel(const float* __restrict__ x, float* __restrict__ y, int P, int H, int W, int Ho, int Wo, int ph, int pw) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)P * Ho * Wo) return;
  const int p = (int)(i / ((long long)Ho * Wo));
  const int rem = (int)(i - (long long)p * Ho * Wo);
  const int r = rem / Wo, c = rem - r * Wo;
  float s = 0.f;
  for (int dy = 0; dy < 2; ++dy)
    for (int dx = 0; dx < 2; ++dx) {
      const int yy = 2 * r - ph + dy, xx = 2 * c - pw + dx;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) s += x[((size_t)p * H + yy) * W + xx];
    }
  y[i] = s * 0.25f;
}

// ms_ssim = mean over planes of prod_l relu(cs_l)^w_l (l < 4) * relu(ssim_4)^w_4
__global__ void ms_final_kernel(const float* __restrict__ ssim, const float* __restrict__ cs, int P, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const float w[MS_LEVELS] = {0.0448f, 0.2856f, 0.3001f, 0.2363f, 0.1333f};
  double acc = 0.0;
  for (int p = 0; p < P; ++p) {
    float v = 1.0f;
    for (int l = 0; l < MS_LEVELS; ++l) {
      const float b = l < MS_LEVELS - 1 ? cs[l * P + p] : ssim[l * P + p];
      v *= powf(fmaxf(b, 0.0f), w[l]);
    }
    acc += (double)v;
  }
  out[0] = (float)(acc / (double)P);
}

// workspace (floats): 2 quantised copies + 2 pyramid buffers of the same size + 2 * 5 * P stats
extern "C" long long tmae_metrics_workspace(int n, int C, int H, int W) {
  const long long numel = (long long)n * C * H * W;
  return 4 * numel + 2 * MS_LEVELS * (long long)n * C + 1024;
}

extern "C" int tmae_image_metrics(const float* org, const float* rec, int n, int C, int H, int W, float* work,
                                  long long work_elems, float* out, void* stream) {
  // out[0] = PSNR (max 255, over the whole batch), out[1] = MS-SSIM (data_range 255, size_average)
  TMAE_REQUIRE(org && rec && work && out && n > 0 && C > 0 && H > 0 && W > 0, "tmae_image_metrics: bad arguments");
  TMAE_REQUIRE(work_elems >= tmae_metrics_workspace(n, C, H, W), "tmae_image_metrics: workspace too small");
  TMAE_REQUIRE(H > (MS_WIN - 1) * 16 && W > (MS_WIN - 1) * 16,
               "tmae_image_metrics: Image size should be larger than %d due to the 4 downsamplings in ms-ssim",
               (MS_WIN - 1) * 16);
  hipStream_t st = (hipStream_t)stream;
  const long long numel = (long long)n * C * H * W;
  const int P = n * C;
  float* qa = work;
  float* qb = qa + numel;
  float* pa = qb + numel;
  float* pb = pa + numel;
  float* ss = pb + numel;
  float* cs = ss + MS_LEVELS * P;
  long long* part = reinterpret_cast<long long*>(cs + MS_LEVELS * P + ((cs + MS_LEVELS * P - work) & 1));
  const unsigned gq = (unsigned)((numel + 255) / 256);
  hipLaunchKernelGGL(quant255_kernel, dim3(gq), dim3(256), 0, st, org, qa, numel);
  hipLaunchKernelGGL(quant255_kernel, dim3(gq), dim3(256), 0, st, rec, qb, numel);
  const int nparts = 256;
  hipLaunchKernelGGL(sqdiff_kernel, dim3(nparts), dim3(256), 0, st, (const float*)qa, (const float*)qb, numel, part);
  hipLaunchKernelGGL(psnr_final_kernel, dim3(1), dim3(64), 0, st, (const long long*)part, nparts, numel, 255.0f, out);
  const MsWin win = ms_window();
  const float c1 = (0.01f * 255.0f) * (0.01f * 255.0f), c2 = (0.03f * 255.0f) * (0.03f * 255.0f);
  const float* x = qa;
  const float* y = qb;
  int h = H, w = W;
  for (int l = 0; l < MS_LEVELS; ++l) {
    hipLaunchKernelGGL(ms_stats_kernel, dim3(P), dim3(256), 0, st, x, y, h, w, win, c1, c2, ss + l * P, cs + l * P);
    if (l < MS_LEVELS - 1) {
      const int ph = h % 2, pw = w % 2;
      const int ho = (h + 2 * ph - 2) / 2 + 1, wo = (w + 2 * pw - 2) / 2 + 1;
      // ping-pong: level l+1 lives in (pa, pb) on even l, in (qa, qb) after that (the quantised copies are
      // no longer needed once level 0 has been measured)
      float* nx = (l % 2 == 0) ? pa : qa;
      float* ny = (l % 2 == 0) ? pb : qb;
      const unsigned g = (unsigned)(((long long)P * ho * wo + 255) / 256);
      hipLaunchKernelGGL(avgpool2_kernel, dim3(g), dim3(256), 0, st, x, nx, P, h, w, ho, wo, ph, pw);
      hipLaunchKernelGGL(avgpool2_kernel, dim3(g), dim3(256), 0, st, y, ny, P, h, w, ho, wo, ph, pw);
      x = nx;
      y = ny;
      h = ho;
      w = wo;
    }
  }
  hipLaunchKernelGGL(ms_final_kernel, dim3(1), dim3(64), 0, st, (const float*)ss, (const float*)cs, P, out + 1);
  TMAE_LAUNCH_CHECK("tmae_image_metrics");
}
