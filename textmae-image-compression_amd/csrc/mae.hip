// MaskedAutoencoderViT pieces that differ from the MCM path (reference models/MAE/models_mae.py):
//
//  * random_masking (models_mae.py:123-148): ids_shuffle = argsort(noise) (ascending, ties by
//    index = a stable sort), ids_restore = argsort(ids_shuffle), binary mask 1 where
//    rank >= len_keep.  One workgroup per image sorts (noise key, index) pairs in LDS.
//  * forward_loss (models_mae.py:198-214): per patch mean((pred - target)^2) over p*p*c, target =
//    patchify(imgs) ("nchpwq -> nhwpqc"), optionally normalised per patch (mean, unbiased var, +1e-6);
//    loss = sum(loss * mask) / sum(mask).  One wave per patch reads its image patch directly (no
//    patchified copy), partial sums in f64 over a fixed grid, folded in index order: deterministic.
#include "sort.h"

#define MAE_MAXL 2048
#define MAE_SORT_THREADS 256

__global__ void __launch_bounds__(MAE_SORT_THREADS)
mae_masking_kernel(const float* __restrict__ noise, int64_t* __restrict__ ids_shuffle, int64_t* __restrict__ ids_restore,
                   float* __restrict__ mask, int L, int P, int keep) {
  __shared__ unsigned long long key[MAE_MAXL];
  const int b = blockIdx.x, t = threadIdx.x;
  const float* s = noise + (size_t)b * L;
  for (int i = t; i < P; i += MAE_SORT_THREADS) {
    if (i < L) {
      float v = s[i];
      if (v == 0.0f) v = 0.0f;  // -0.0 == 0.0
      key[i] = ((unsigned long long)f2key(v) << 32) | (unsigned)i;
    } else {
      key[i] = ~0ull;
    }
  }
  __syncthreads();
  lds_bitonic_sort<MAE_SORT_THREADS>(key, P);
  for (int r = t; r < L; r += MAE_SORT_THREADS) {
    const int idx = (int)(key[r] & 0xffffffffu);
    ids_shuffle[(size_t)b * L + r] = idx;
    ids_restore[(size_t)b * L + idx] = r;
    if (mask) mask[(size_t)b * L + idx] = r >= keep ? 1.0f : 0.0f;
  }
}

extern "C" int tmae_mae_masking(const float* noise, int64_t* ids_shuffle, int64_t* ids_restore, float* mask, int n,
                                int L, int keep, void* stream) {
  TMAE_REQUIRE(noise && ids_shuffle && ids_restore && n >= 0 && L >= 1 && L <= MAE_MAXL,
               "tmae_mae_masking: L=%d must be in [1, %d]", L, MAE_MAXL);
  TMAE_REQUIRE(keep >= 0 && keep <= L, "tmae_mae_masking: len_keep=%d outside [0, %d]", keep, L);
  if (n == 0) return TMAE_OK;
  int P = 1;
  while (P < L) P <<= 1;
  hipLaunchKernelGGL(mae_masking_kernel, dim3(n), dim3(MAE_SORT_THREADS), 0, (hipStream_t)stream, noise, ids_shuffle,
                     ids_restore, mask, L, P, keep);
  TMAE_LAUNCH_CHECK("tmae_mae_masking");
}

// ------------------------------------------------------------------ masked MSE
#define MAE_LOSS_BLOCKS 512
#define MAE_VPL 32  // values per lane held in registers: p*p*c <= 64 * 32 = 2048

__device__ __forceinline__ float wave_sum(float v) { return wave_allsum(v); }

// offset of value lane + 64 k of a patchified row (e = (py * P + px) * C + c) from the patch's top-left pixel in
// plane 0 of its image (NCHW), -1 past the row: the same for every row, so worked out once per thread (the two
// integer divisions per value were most of the loss kernels' time)
__device__ __forceinline__ void mae_offsets(int P, int C, int H, int W, int lane, int (&off)[MAE_VPL]) {
  const int D = P * P * C;
#pragma unroll
  for (int k = 0; k < MAE_VPL; ++k) {
    const int e = lane + 64 * k;
    const int q = e / C, c = e - q * C;
    const int py = q / P, px = q - py * P;
    off[k] = e < D ? (c * H + py) * W + px : -1;
  }
}

// the target of patch `row` (= b * L + l) in the lane-strided layout t[k] = value lane + 64 k of the patchified row
// (models_mae.py:198-214 patchify + norm_pix_loss), offsets from mae_offsets
__device__ __forceinline__ void mae_target(const float* __restrict__ imgs, int row, int L, int G, int P, int C, int H,
                                           int W, int norm_pix, int lane, const int (&off)[MAE_VPL], float (&t)[MAE_VPL]) {
  const int D = P * P * C;
  const int b = row / L, l = row - b * L;
  const int hy = l / G, hx = l - hy * G;
  const float* img = imgs + (size_t)b * C * H * W + (size_t)(hy * P) * W + hx * P;
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < MAE_VPL; ++k) {
    t[k] = off[k] >= 0 ? img[off[k]] : 0.0f;
    s += t[k];
  }
  if (norm_pix) {
    const float mean = wave_sum(s) / (float)D;
    float v = 0.0f;
#pragma unroll
    for (int k = 0; k < MAE_VPL; ++k)
      if (off[k] >= 0) v += (t[k] - mean) * (t[k] - mean);
    const float var = wave_sum(v) / (float)(D - 1);
    const float inv = 1.0f / sqrtf(var + 1e-6f);
#pragma unroll
    for (int k = 0; k < MAE_VPL; ++k) t[k] = (t[k] - mean) * inv;
  }
}

// PC / CC: the patch size / channel count as compile-time constants (16 / 3: every bench and reference config),
// 0 = the run-time values; the constants turn mae_offsets' divisions into multiplies
template <int PC, int CC>
__global__ void __launch_bounds__(256)
mae_loss_partial_kernel(const float* __restrict__ pred, const float* __restrict__ imgs,
                        const int64_t* __restrict__ ids_restore, int n, int L, int G, int P_, int C_, int H, int W,
                        int keep, int norm_pix, double* __restrict__ part) {
  const int P = PC ? PC : P_, C = CC ? CC : C_;
  __shared__ double red[2][4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D = P * P * C;
  double num = 0.0, den = 0.0;
  int off[MAE_VPL];
  mae_offsets(P, C, H, W, lane, off);
  for (int row = blockIdx.x * 4 + wave; row < n * L; row += gridDim.x * 4) {
    const int b = row / L, l = row - b * L;
    float t[MAE_VPL];
    mae_target(imgs, row, L, G, P, C, H, W, norm_pix, lane, off, t);
    const float* pr = pred + (size_t)row * D;
    float se = 0.0f;
#pragma unroll
    for (int k = 0; k < MAE_VPL; ++k) {
      const int e = lane + 64 * k;
      if (e < D) {
        const float d = pr[e] - t[k];
        se += d * d;
      }
    }
    const float patch_loss = wave_sum(se) / (float)D;
    const float m = ids_restore[(size_t)b * L + l] >= keep ? 1.0f : 0.0f;
    num += (double)(patch_loss * m);
    den += (double)m;
  }
  if (lane == 0) {
    red[0][wave] = num;
    red[1][wave] = den;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[2 * blockIdx.x + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

__global__ void __launch_bounds__(256) mae_loss_final_kernel(const double* __restrict__ part, int np,
                                                             float* __restrict__ out) {
  __shared__ double red[2][256];
  double a = 0.0, c = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) {
    a += part[2 * i];
    c += part[2 * i + 1];
  }
  red[0][threadIdx.x] = a;
  red[1][threadIdx.x] = c;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0][0] / red[1][0]);
}

// pred: [n*L][P*P*C] f32; imgs NCHW f32; ids_restore [n][L]; work: >= 2 * 512 doubles
extern "C" int tmae_mae_loss(const float* pred, const float* imgs, const int64_t* ids_restore, int n, int C, int H,
                             int W, int P, int keep, int norm_pix_loss, double* work, float* out, void* stream) {
  TMAE_REQUIRE(pred && imgs && ids_restore && work && out && P > 0 && H % P == 0 && W == H,
               "tmae_mae_loss: bad arguments (H=%d W=%d P=%d)", H, W, P);
  TMAE_REQUIRE(P * P * C <= 64 * MAE_VPL && P * P * C > 1, "tmae_mae_loss: patch of %d values unsupported", P * P * C);
  const int G = H / P, L = G * G;
  hipStream_t st = (hipStream_t)stream;
  if (P == 16 && C == 3)
    hipLaunchKernelGGL((mae_loss_partial_kernel<16, 3>), dim3(MAE_LOSS_BLOCKS), dim3(256), 0, st, pred, imgs,
                       ids_restore, n, L, G, P, C, H, W, keep, norm_pix_loss, work);
  else
    hipLaunchKernelGGL((mae_loss_partial_kernel<0, 0>), dim3(MAE_LOSS_BLOCKS), dim3(256), 0, st, pred, imgs,
                       ids_restore, n, L, G, P, C, H, W, keep, norm_pix_loss, work);
  hipLaunchKernelGGL(mae_loss_final_kernel, dim3(1), dim3(256), 0, st, work, MAE_LOSS_BLOCKS, out);
  TMAE_LAUNCH_CHECK("tmae_mae_loss");
}

// ------------------------------------------------------------------ masked MSE backward
// d loss / d pred[b][l][e] = g * mask[b][l] * 2 (pred - target) / (D * sum(mask)), sum(mask) = n (L - len_keep)
// (autograd of models_mae.py:212-214); plus an incoming gradient of pred itself when dpred_in is given.
// One wave per patch row, written in the operand dtype of the decoder_pred weight / data gradients.
template <typename OT, int PC, int CC>
__global__ void __launch_bounds__(256)
mae_loss_bwd_kernel(const float* __restrict__ pred, const float* __restrict__ imgs, const int64_t* __restrict__ ids_restore,
                    int n, int L, int G, int P_, int C_, int H, int W, int keep, int norm_pix, const float* __restrict__ dloss,
                    const float* __restrict__ dpred_in, OT* __restrict__ out) {
  const int P = PC ? PC : P_, C = CC ? CC : C_;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int D = P * P * C;
  const float msum = (float)n * (float)(L - keep);
  const float g = dloss ? dloss[0] : 0.0f;
  int off[MAE_VPL];
  mae_offsets(P, C, H, W, lane, off);
  for (int row = blockIdx.x * 4 + wave; row < n * L; row += gridDim.x * 4) {
    const float m = ids_restore[row] >= keep ? 1.0f : 0.0f;
    const float sc = m > 0.0f && msum > 0.0f ? g * m / msum / (float)D : 0.0f;
    const float* pr = pred + (size_t)row * D;
    OT* o = out + (size_t)row * D;
    const float* di = dpred_in ? dpred_in + (size_t)row * D : nullptr;
    float t[MAE_VPL];
    if (sc != 0.0f) mae_target(imgs, row, L, G, P, C, H, W, norm_pix, lane, off, t);
#pragma unroll
    for (int k = 0; k < MAE_VPL; ++k) {
      const int e = lane + 64 * k;
      if (e < D) {
        float v = sc != 0.0f ? 2.0f * (pr[e] - t[k]) * sc : 0.0f;
        if (di) v += di[e];
        o[e] = (OT)v;
      }
    }
  }
}

extern "C" int tmae_mae_loss_bwd(const float* pred, const float* imgs, const int64_t* ids_restore, int n, int C, int H,
                                 int W, int P, int keep, int norm_pix_loss, const float* dloss, const float* dpred_in,
                                 void* out, int out_dtype, void* stream) {
  TMAE_REQUIRE(pred && imgs && ids_restore && out && P > 0 && H % P == 0 && W == H,
               "tmae_mae_loss_bwd: bad arguments (H=%d W=%d P=%d)", H, W, P);
  TMAE_REQUIRE(P * P * C <= 64 * MAE_VPL && P * P * C > 1, "tmae_mae_loss_bwd: patch of %d values unsupported",
               P * P * C);
  TMAE_REQUIRE(out_dtype == TMAE_F32 || out_dtype == TMAE_BF16, "tmae_mae_loss_bwd: out dtype %d", out_dtype);
  const int G = H / P, L = G * G;
  if (n == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  // about three rows per wave: the per-thread offset table is worked out once per wave
  const int nb = ceil_div(n * L, 12);
  const dim3 grid((unsigned)(nb < 2048 ? nb : 2048));
#define MAE_BWD_LAUNCH(OT, PC, CC)                                                                                   \
  hipLaunchKernelGGL((mae_loss_bwd_kernel<OT, PC, CC>), grid, dim3(256), 0, st, pred, imgs, ids_restore, n, L, G, P, C, \
                     H, W, keep, norm_pix_loss, dloss, dpred_in, (OT*)out)
  const bool std_patch = P == 16 && C == 3;
  if (out_dtype == TMAE_BF16) {
    if (std_patch) MAE_BWD_LAUNCH(bf16, 16, 3);
    else MAE_BWD_LAUNCH(bf16, 0, 0);
  } else {
    if (std_patch) MAE_BWD_LAUNCH(float, 16, 3);
    else MAE_BWD_LAUNCH(float, 0, 0);
  }
#undef MAE_BWD_LAUNCH
  TMAE_LAUNCH_CHECK("tmae_mae_loss_bwd");
}
