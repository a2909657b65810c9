// VGG16 feature loss of MCM.forward_loss (reference models/Compression/loss/vgg.py:86-115, called from
// MCM.py:711): de_normalize + normalize_batch (common/image_utils.py:4-23), VGG16 features[0:16]
// (relu1_2 / relu2_2 / relu3_3 slices, torchvision layout), MSE(relu2_2) + MSE(relu3_3).
// The 3x3 convolutions (+ ReLU in the epilogue) and their data gradients are the library's conv kernels
// (tmae_conv3x3 with TMAE_ACT_RELU, tmae_conv_dgrad); this file holds the glue, all NHWC:
//   prep      NCHW f32 image -> NHWC operand with the channel count padded to 8 (zero channels)
//   maxpool   2x2 stride 2 with the argmax kept for the backward (first maximum wins, as torch's)
//   relu mask dz = dy * (y > 0)
//   mse       mean((a - b)^2) in fixed-grid f64 partial sums, and its gradient 2 (a - b) / numel * g
//   prep bwd  the NHWC input gradient back to NCHW f32 (3 channels), through the normalisation
#include "common.h"

#define VGG_BLOCKS 1024

__constant__ float kVggMean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float kVggStd[3] = {0.229f, 0.224f, 0.225f};

template <typename T>
__global__ void __launch_bounds__(256) vgg_prep_kernel(const float* __restrict__ x, T* __restrict__ y, int n, int C,
                                                       int HW, int CP) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * HW * CP) return;
  const int c = (int)(i % CP);
  const long long p = i / CP;
  const int b = (int)(p / HW), pix = (int)(p - (long long)b * HW);
  float v = 0.0f;
  if (c < C) {
    // (x + 1) / 2 * 255, / 255, - mean, / std: the reference's op order (f32 throughout)
    float t = (x[((size_t)b * C + c) * HW + pix] + 1.0f) / 2.0f * 255.0f;
    t = t / 255.0f;
    t = t - kVggMean[c];
    v = t / kVggStd[c];
  }
  y[i] = to_out<T>(v);
}

template <typename T>
__global__ void __launch_bounds__(256) vgg_prep_bwd_kernel(const T* __restrict__ g, float* __restrict__ dx, int n, int C,
                                                           int HW, int CP) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * C * HW) return;
  const int pix = (int)(i % HW);
  const long long bc = i / HW;
  const int c = (int)(bc % C), b = (int)(bc / C);
  float v = (float)g[((size_t)b * HW + pix) * CP + c];
  v = v / kVggStd[c];
  v = v / 255.0f;
  v = v * 255.0f;
  dx[i] = v / 2.0f;
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool2_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                       unsigned char* __restrict__ arg, int n, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2;
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * Ho * Wo * C) return;
  const int c = (int)(i % C);
  const long long p = i / C;
  const int wo = (int)(p % Wo);
  const long long q = p / Wo;
  const int ho = (int)(q % Ho), b = (int)(q / Ho);
  float best = -INFINITY;
  int bi = 0;
  for (int k = 0; k < 4; ++k) {
    const int yy = 2 * ho + (k >> 1), xx = 2 * wo + (k & 1);
    const float v = (float)x[(((size_t)b * H + yy) * W + xx) * C + c];
    if (v > best || v != v) {  // torch max_pool2d: strict '>' (first maximum wins), NaN propagates
      best = v;
      bi = k;
    }
  }
  y[i] = to_out<T>(best);
  if (arg) arg[i] = (unsigned char)bi;
}

template <typename T>
__global__ void __launch_bounds__(256) maxpool2_bwd_kernel(const T* __restrict__ dy, const unsigned char* __restrict__ arg,
                                                           T* __restrict__ dx, int n, int H, int W, int C,
                                                           const T* __restrict__ add) {
  // dx [n][H][W][C] (every element written: 0 off the argmax), optionally + add (a second gradient source)
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * H * W * C) return;
  const int c = (int)(i % C);
  const long long p = i / C;
  const int x = (int)(p % W);
  const long long q = p / W;
  const int y = (int)(q % H), b = (int)(q / H);
  const int Ho = H / 2, Wo = W / 2;
  const int ho = y >> 1, wo = x >> 1, k = ((y & 1) << 1) | (x & 1);
  float v = 0.0f;
  if (ho < Ho && wo < Wo) {
    const size_t o = (((size_t)b * Ho + ho) * Wo + wo) * C + c;
    if (arg[o] == k) v = (float)dy[o];
  }
  if (add) v += (float)add[i];
  dx[i] = to_out<T>(v);
}

template <typename T>
__global__ void __launch_bounds__(256) relu_mask_kernel(T* __restrict__ g, const T* __restrict__ y, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n && !((float)y[i] > 0.0f)) g[i] = to_out<T>(0.0f);
}

template <typename T>
__global__ void __launch_bounds__(256) mse_part_kernel(const T* __restrict__ a, const T* __restrict__ b, long long n,
                                                       double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float d = (float)a[i] - (float)b[i];
    s += (double)(d * d);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void mse_final_kernel(const double* __restrict__ part, int nparts, double inv_n, float* __restrict__ out,
                                 int accumulate) {
  if (threadIdx.x != 0) return;
  double s = 0.0;
  for (int i = 0; i < nparts; ++i) s += part[i];
  const float v = (float)(s * inv_n);
  out[0] = accumulate ? out[0] + v : v;
}

template <typename T>
__global__ void __launch_bounds__(256) mse_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b, long long n,
                                                      const float* __restrict__ g, float scale, T* __restrict__ da) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) da[i] = to_out<T>(g[0] * (scale * ((float)a[i] - (float)b[i])));
}

static inline unsigned grid_of(long long n) { return (unsigned)((n + 255) / 256); }

extern "C" int tmae_vgg_prep(const float* x, int n, int C, int H, int W, int CP, void* y, int dtype, void* stream) {
  TMAE_REQUIRE(x && y && C <= 3 && CP >= C, "tmae_vgg_prep: bad arguments");
  const long long tot = (long long)n * H * W * CP;
  if (tot == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(vgg_prep_kernel<bf16>, dim3(grid_of(tot)), dim3(256), 0, st, x, (bf16*)y, n, C, H * W, CP);
  else
    hipLaunchKernelGGL(vgg_prep_kernel<float>, dim3(grid_of(tot)), dim3(256), 0, st, x, (float*)y, n, C, H * W, CP);
  TMAE_LAUNCH_CHECK("tmae_vgg_prep");
}

extern "C" int tmae_vgg_prep_bwd(const void* g, int n, int C, int H, int W, int CP, float* dx, int dtype, void* stream) {
  TMAE_REQUIRE(g && dx && C <= 3 && CP >= C, "tmae_vgg_prep_bwd: bad arguments");
  const long long tot = (long long)n * C * H * W;
  if (tot == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(vgg_prep_bwd_kernel<bf16>, dim3(grid_of(tot)), dim3(256), 0, st, (const bf16*)g, dx, n, C, H * W, CP);
  else
    hipLaunchKernelGGL(vgg_prep_bwd_kernel<float>, dim3(grid_of(tot)), dim3(256), 0, st, (const float*)g, dx, n, C,
                       H * W, CP);
  TMAE_LAUNCH_CHECK("tmae_vgg_prep_bwd");
}

extern "C" int tmae_maxpool2(const void* x, int n, int H, int W, int C, void* y, unsigned char* arg, int dtype,
                             void* stream) {
  TMAE_REQUIRE(x && y && H % 2 == 0 && W % 2 == 0, "tmae_maxpool2: needs even H, W (got %d x %d)", H, W);
  const long long tot = (long long)n * (H / 2) * (W / 2) * C;
  if (tot == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(maxpool2_kernel<bf16>, dim3(grid_of(tot)), dim3(256), 0, st, (const bf16*)x, (bf16*)y, arg, n, H,
                       W, C);
  else
    hipLaunchKernelGGL(maxpool2_kernel<float>, dim3(grid_of(tot)), dim3(256), 0, st, (const float*)x, (float*)y, arg, n,
                       H, W, C);
  TMAE_LAUNCH_CHECK("tmae_maxpool2");
}

extern "C" int tmae_maxpool2_bwd(const void* dy, const unsigned char* arg, int n, int H, int W, int C, void* dx,
                                 const void* add, int dtype, void* stream) {
  TMAE_REQUIRE(dy && arg && dx && H % 2 == 0 && W % 2 == 0, "tmae_maxpool2_bwd: bad arguments");
  const long long tot = (long long)n * H * W * C;
  if (tot == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<bf16>, dim3(grid_of(tot)), dim3(256), 0, st, (const bf16*)dy, arg, (bf16*)dx, n,
                       H, W, C, (const bf16*)add);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(grid_of(tot)), dim3(256), 0, st, (const float*)dy, arg,
                       (float*)dx, n, H, W, C, (const float*)add);
  TMAE_LAUNCH_CHECK("tmae_maxpool2_bwd");
}

extern "C" int tmae_relu_mask(void* g, const void* y, long long n, int dtype, void* stream) {
  TMAE_REQUIRE(g && y, "tmae_relu_mask: bad arguments");
  if (n <= 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(relu_mask_kernel<bf16>, dim3(grid_of(n)), dim3(256), 0, st, (bf16*)g, (const bf16*)y, n);
  else
    hipLaunchKernelGGL(relu_mask_kernel<float>, dim3(grid_of(n)), dim3(256), 0, st, (float*)g, (const float*)y, n);
  TMAE_LAUNCH_CHECK("tmae_relu_mask");
}

// out[0] (+)= mean((a - b)^2); part >= VGG_BLOCKS doubles
extern "C" int tmae_mse(const void* a, const void* b, long long n, double* part, float* out, int accumulate, int dtype,
                        void* stream) {
  TMAE_REQUIRE(a && b && part && out && n > 0, "tmae_mse: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)std::min<long long>(VGG_BLOCKS, (n + 255) / 256);
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(mse_part_kernel<bf16>, dim3(nb), dim3(256), 0, st, (const bf16*)a, (const bf16*)b, n, part);
  else
    hipLaunchKernelGGL(mse_part_kernel<float>, dim3(nb), dim3(256), 0, st, (const float*)a, (const float*)b, n, part);
  hipLaunchKernelGGL(mse_final_kernel, dim3(1), dim3(64), 0, st, (const double*)part, nb, 1.0 / (double)n, out,
                     accumulate);
  TMAE_LAUNCH_CHECK("tmae_mse");
}

// da = g[0] * 2 (a - b) / n  (MSELoss backward w.r.t. its first input)
extern "C" int tmae_mse_bwd(const void* a, const void* b, long long n, const float* g, void* da, int dtype, void* stream) {
  TMAE_REQUIRE(a && b && g && da && n > 0, "tmae_mse_bwd: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const float scale = (float)(2.0 / (double)n);
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(mse_bwd_kernel<bf16>, dim3(grid_of(n)), dim3(256), 0, st, (const bf16*)a, (const bf16*)b, n, g,
                       scale, (bf16*)da);
  else
    hipLaunchKernelGGL(mse_bwd_kernel<float>, dim3(grid_of(n)), dim3(256), 0, st, (const float*)a, (const float*)b, n, g,
                       scale, (float*)da);
  TMAE_LAUNCH_CHECK("tmae_mse_bwd");
}
