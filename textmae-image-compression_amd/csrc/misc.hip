// Small data-movement kernels around the GEMMs, plus the library's error plumbing.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

// ------------------------------------------------------------------ error state (thread-local)
static thread_local char g_err[512] = "";

void tmae_set_error(int code, const char* fmt, ...) {
  (void)code;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* tmae_last_error_string(void) { return g_err; }
extern "C" int tmae_abi_version(void) { return TMAE_ABI_VERSION; }

// ------------------------------------------------------------------ cls rows
// tokens[b][0][:] = cls_token + pos[0]   (MCM.py:624-626 / models_mae.py forward_encoder)
__global__ void cls_rows_kernel(float* __restrict__ tok, const float* __restrict__ cls, const float* __restrict__ pos,
                                int n, int rows_per_img, int D) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * D) return;
  const int b = i / D, d = i - b * D;
  tok[(size_t)b * rows_per_img * D + d] = cls[d] + pos[d];
}

extern "C" int tmae_cls_rows(float* tokens, const float* cls, const float* pos, int n, int rows_per_img, int D,
                             void* stream) {
  if (n * D == 0) return TMAE_OK;
  hipLaunchKernelGGL(cls_rows_kernel, dim3(ceil_div(n * D, 256)), dim3(256), 0, (hipStream_t)stream, tokens, cls, pos,
                     n, rows_per_img, D);
  TMAE_LAUNCH_CHECK("tmae_cls_rows");
}

// ------------------------------------------------------------------ decoder mask-token rows
// For kept ranks m in [ntok-1, L): decoder row 1 + ids_shuffle[b][m] = mask_token + pos[row]
// (MCM.py:660-675: the mask tokens land wherever ids_restore points past the kept tokens).
__global__ void mask_rows_kernel(float* __restrict__ out, const float* __restrict__ mask,
                                 const float* __restrict__ pos, const int64_t* __restrict__ ids, int n, int L,
                                 int ntok, int D) {
  const int nm = L - (ntok - 1);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int per_img = nm * (D / 4);
  if (i >= n * per_img) return;
  const int b = i / per_img, rem = i - b * per_img;
  const int mi = rem / (D / 4), d = 4 * (rem - mi * (D / 4));
  const int row = 1 + (int)ids[(size_t)b * L + (ntok - 1) + mi];
  const f32x4 v = load4f(mask + d) + load4f(pos + (size_t)row * D + d);
  store4(out + ((size_t)b * (L + 1) + row) * D + d, v);
}

extern "C" int tmae_mask_rows(float* out, const float* mask_token, const float* pos, const int64_t* ids_shuffle,
                              int n, int L, int ntok, int D, void* stream) {
  TMAE_REQUIRE(D % 4 == 0 && ntok >= 1 && ntok <= L + 1, "tmae_mask_rows: bad shape");
  const int total = n * (L - (ntok - 1)) * (D / 4);
  if (total <= 0) return TMAE_OK;
  hipLaunchKernelGGL(mask_rows_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, out, mask_token,
                     pos, ids_shuffle, n, L, ntok, D);
  TMAE_LAUNCH_CHECK("tmae_mask_rows");
}

// ------------------------------------------------------------------ NHWC -> NCHW (fp32)
__global__ void nhwc_to_nchw_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y, int n, int C, int HW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * C * HW) return;
  const int pix = i % HW, t = i / HW;
  const int c = t % C, b = t / C;
  y[i] = x[((size_t)b * HW + pix) * ldx + c];
}

extern "C" int tmae_nhwc_to_nchw(const float* x, int ldx, float* y, int n, int C, int HW, void* stream) {
  const int total = n * C * HW;
  if (total <= 0) return TMAE_OK;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(ceil_div(total, 256)), dim3(256), 0, (hipStream_t)stream, x, ldx, y, n,
                     C, HW);
  TMAE_LAUNCH_CHECK("tmae_nhwc_to_nchw");
}

// ------------------------------------------------------------------ rate (bits per pixel)
// RateDistortionLoss bpp term (reference models/Compression/loss/rd_loss.py:19-20):
//   sum over both likelihood tensors of log(lik) / (-ln 2 * N*H*W)
// Two deterministic passes: per-block partial sums in f64 (fixed grid), then one block folds them
// in index order, so the result does not depend on scheduling.
#define BPP_BLOCKS 512

__global__ void __launch_bounds__(256)
log_sum_partial_kernel(const float* __restrict__ a, long long na, const float* __restrict__ b, long long nb,
                       double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const long long total = na + nb;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const float v = i < na ? a[i] : b[i - na];
    s += (double)logf(v);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) log_sum_final_kernel(const double* __restrict__ part, int np, double scale,
                                                            float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] * scale);
}

extern "C" int tmae_bpp_sum(const float* y_lik, long long ny, const float* z_lik, long long nz, double* work,
                            float* out, double num_pixels, void* stream) {
  TMAE_REQUIRE(work != nullptr && out != nullptr && num_pixels > 0, "tmae_bpp_sum: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(log_sum_partial_kernel, dim3(BPP_BLOCKS), dim3(256), 0, st, y_lik, ny, z_lik, nz, work);
  hipLaunchKernelGGL(log_sum_final_kernel, dim3(1), dim3(256), 0, st, work, BPP_BLOCKS,
                     1.0 / (-0.69314718055994530942 * num_pixels), out);
  TMAE_LAUNCH_CHECK("tmae_bpp_sum");
}

// ------------------------------------------------------------------ training-set random crops
// The training loader's per-sample work on a DIV2K-shaped set (training.py:115-129 builds the loader;
// utils/dataloader.py:58-61: ToTensor then Normalize): crop S x S from a uint8 HWC image, x = v / 255, then
// (x - mean) / std per channel, into NCHW f32.  Same f32 operations in the same order as torchvision's
// ToTensor (div 255) and Normalize (sub mean, div std), so the result is bitwise torch's.
// crops[b] = (source image, top, left).  One thread per output pixel: 3 byte loads, 3 coalesced plane stores.
__global__ void crop_normalize_u8_kernel(const unsigned char* __restrict__ src, int H, int W,
                                         const int* __restrict__ crops, int B, int S, float m0, float m1, float m2,
                                         float s0, float s1, float s2, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)S * S;
  if (i >= (long long)B * per) return;
  const int b = (int)(i / per);
  const int p = (int)(i - (long long)b * per), y = p / S, x = p - y * S;
  const int img = crops[3 * b], top = crops[3 * b + 1], left = crops[3 * b + 2];
  const unsigned char* px = src + (((size_t)img * H + top + y) * W + left + x) * 3;
  float* o = out + (size_t)b * 3 * per + p;
  o[0] = (px[0] / 255.0f - m0) / s0;
  o[per] = (px[1] / 255.0f - m1) / s1;
  o[2 * per] = (px[2] / 255.0f - m2) / s2;
}

extern "C" int tmae_crop_normalize_u8(const unsigned char* src, int nsrc, int H, int W, const int* crops, int B,
                                      int S, const float* mean, const float* std, float* out, void* stream) {
  TMAE_REQUIRE(nsrc > 0 && S > 0 && S <= H && S <= W, "tmae_crop_normalize_u8: crop %d exceeds the %dx%d images", S,
               H, W);
  TMAE_REQUIRE(mean != nullptr && std != nullptr, "tmae_crop_normalize_u8: mean / std are NULL");
  const long long total = (long long)B * S * S;
  if (total == 0) return TMAE_OK;
  hipLaunchKernelGGL(crop_normalize_u8_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, src, H, W, crops, B, S, mean[0], mean[1], mean[2], std[0], std[1], std[2],
                     out);
  TMAE_LAUNCH_CHECK("tmae_crop_normalize_u8");
}
