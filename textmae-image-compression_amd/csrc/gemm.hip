// MFMA GEMM family for gfx950: every dense contraction on the hot path.
//
//   out[m][n] = epilogue( sum_k X[m][k] * W[n][k] + bias[n] )
//
// W is always a [N][K] row-major weight (nn.Linear layout; conv weights are re-laid out to
// [Cout][ky][kx][Cin] once at weight-prep time).  X rows come from a "row loader": plain dense
// rows, an implicit-GEMM 3x3 conv gather over NHWC activations, or the patch-embed gather over
// the NCHW image restricted to the KEPT patches (masking happens before the embedding, so the
// 112 masked patches of each image are never multiplied).
//
// Tiling (cdna_hip_programming.md §5): 256 threads = 4 waves, tile BN x BM, K-tile = 128 bytes
// per row (64 bf16 or 32 f32).  Global -> registers -> LDS (double buffered, one barrier per
// K-tile, next tile's global loads issued before the current tile's MFMAs).  LDS rows are 128 B
// with the 16-B chunk XOR-swizzled by ((row >> 1) & 7), which makes the ds_read_b128 fragment reads
// conflict-free for 16 consecutive rows.  The MFMA is issued "swapped" (A = weight rows,
// B = activation rows) so each lane ends up owning 4 CONSECUTIVE output columns of one output
// row: 16-B (f32) / 8-B (bf16) epilogue stores.
//   bf16: v_mfma_f32_16x16x32_bf16, f32 accumulate (throughput path)
//   f32 : v_mfma_f32_16x16x4_f32 (exact f32 fma chain; the parity path)
#include "common.h"

template <typename T> struct Elt;
template <> struct Elt<bf16> { static constexpr int EPC = 8; };
template <> struct Elt<float> { static constexpr int EPC = 4; };

// ------------------------------------------------------------------ chunk conversion
template <typename T> __device__ __forceinline__ uint4 load_chunk_from_f32(const float* p);
template <> __device__ __forceinline__ uint4 load_chunk_from_f32<float>(const float* p) {
  return *reinterpret_cast<const uint4*>(p);
}
template <> __device__ __forceinline__ uint4 load_chunk_from_f32<bf16>(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  return pack8_bf16(a, b);
}

// ------------------------------------------------------------------ row loaders
// Dense rows of S (= T, or float converted to T).  Row remap for strided views:
//   source row = (m / G) * Gs + off + (m % G)
template <typename T, typename S> struct DenseRows {
  const S* p;
  int ld, rows, K, G, Gs, off;
  struct Row { const S* ptr; };
  struct Col { int k; bool ok; };
  __device__ Row row(int m) const {
    if (m >= rows) return {nullptr};
    const int sm = (m / G) * Gs + off + (m % G);
    return {p + (size_t)sm * ld};
  }
  __device__ Col col(int kc) const {
    const int k = kc * Elt<T>::EPC;
    return {k, k < K};
  }
  __device__ uint4 load(const Row& r, const Col& c) const {
    if (!r.ptr || !c.ok) return uint4{0, 0, 0, 0};
    if constexpr (sizeof(S) == sizeof(T)) return *reinterpret_cast<const uint4*>(r.ptr + c.k);
    else return load_chunk_from_f32<T>(reinterpret_cast<const float*>(r.ptr) + c.k);
  }
};

// Implicit-GEMM 3x3 conv (padding 1, stride s) over fp32 NHWC activations, input channels
// split over two segments (channel concat without a copy: MCM.py:761,766,780 torch.cat).
// K index = (ky*3 + kx) * Cin + c.
template <typename T> struct ConvRows {
  const float* x1;
  const float* x2;
  int c1, ld1, ld2, Cin, H, W, Ho, Wo, stride, rows, K;
  float inv_cin;
  struct Row { int pix; int iy0; int ix0; bool ok; };
  struct Col { int ky; int kx; int c; bool ok; };
  __device__ Row row(int m) const {
    if (m >= rows) return {0, 0, 0, false};
    const int hw = Ho * Wo;
    const int b = m / hw, rem = m - b * hw;
    const int oy = rem / Wo, ox = rem - oy * Wo;
    return {b * H * W, oy * stride - 1, ox * stride - 1, true};
  }
  __device__ Col col(int kc) const {
    const int k = kc * Elt<T>::EPC;
    if (k >= K) return {0, 0, 0, false};
    int tap = (int)((float)k * inv_cin);
    if (tap * Cin > k) --tap;
    if ((tap + 1) * Cin <= k) ++tap;
    const int c = k - tap * Cin;
    const int ky = tap / 3;
    return {ky, tap - ky * 3, c, true};
  }
  __device__ uint4 load(const Row& r, const Col& c) const {
    const int iy = r.iy0 + c.ky, ix = r.ix0 + c.kx;
    if (!r.ok || !c.ok || iy < 0 || iy >= H || ix < 0 || ix >= W) return uint4{0, 0, 0, 0};
    const int pix = r.pix + iy * W + ix;
    const float* src = (c.c < c1) ? x1 + (size_t)pix * ld1 + c.c : x2 + (size_t)pix * ld2 + (c.c - c1);
    return load_chunk_from_f32<T>(src);
  }
};

// Patch-embed gather (timm PatchEmbed conv16/s16 as a GEMM, MCM.py:615) over the kept patches:
// GEMM row m = (image b, kept rank k) reads patch p = ids_shuffle[b][k] of the NCHW fp32 image.
// K index = c*P*P + py*P + px (conv weight flatten order).
template <typename T> struct PatchRows {
  const float* img;
  const int64_t* ids;
  int L, keep, C, H, W, P, G, rows, K;
  struct Row { const float* base; };
  struct Col { int off; bool ok; };
  __device__ Row row(int m) const {
    if (m >= rows) return {nullptr};
    const int b = m / keep, k = m - b * keep;
    const int p = (int)ids[(size_t)b * L + k];
    const int hy = p / G, hx = p - hy * G;
    return {img + (size_t)b * C * H * W + (size_t)(hy * P) * W + hx * P};
  }
  __device__ Col col(int kc) const {
    const int k = kc * Elt<T>::EPC;
    if (k >= K) return {0, false};
    const int pp = P * P;
    const int c = k / pp, rem = k - c * pp;
    const int py = rem / P, px = rem - py * P;
    return {(c * H + py) * W + px, true};
  }
  __device__ uint4 load(const Row& r, const Col& c) const {
    if (!r.base || !c.ok) return uint4{0, 0, 0, 0};
    return load_chunk_from_f32<T>(r.base + c.off);
  }
};

// ------------------------------------------------------------------ epilogues
// Each receives (m, n, v) with v = 4 accumulators for output columns n..n+3 (n % 4 == 0).
template <typename OT, int ACT> struct EpiStore {
  OT* out;
  int ldo;
  const float* bias;
  __device__ void operator()(int m, int n, f32x4 v) const {
    if (bias) v += load4f(bias + n);
    if (ACT == TMAE_ACT_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_erf(v[j]);
    }
    store4(out + (size_t)m * ldo + n, v);
  }
};

// residual stream update x += W·a + b (timm Block residual adds)
struct EpiResidual {
  float* out;
  int ldo;
  const float* bias;
  __device__ void operator()(int m, int n, f32x4 v) const {
    float* p = out + (size_t)m * ldo + n;
    f32x4 r = load4f(p);
    if (bias) v += load4f(bias + n);
    // reference order: x + (proj(out) ) where proj = acc + bias
    store4(p, r + v);
  }
};

// patch embed: token row b*(keep+1) + 1 + k  <-  acc + bias + pos[1 + p]   (MCM.py:615-626)
struct EpiPatchEmbed {
  float* tok;
  const float* bias;
  const float* pos;
  const int64_t* ids;
  int L, keep, D;
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int b = m / keep, k = m - b * keep;
    const int p = (int)ids[(size_t)b * L + k];
    v += load4f(bias + n);
    v += load4f(pos + (size_t)(1 + p) * D + n);
    store4(tok + ((size_t)b * (keep + 1) + 1 + k) * D + n, v);
  }
};

// decoder embed + unshuffle (MCM.py:657-675; also models_mae.py forward_decoder):
// token k of image b goes to decoder row 0 if k == 0, else row 1 + ids_shuffle[b][k-1]; + pos.
struct EpiDecoderEmbed {
  float* out;
  const float* bias;
  const float* pos;
  const int64_t* ids;
  int L, ntok, D;
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int b = m / ntok, k = m - b * ntok;
    const int row = (k == 0) ? 0 : 1 + (int)ids[(size_t)b * L + (k - 1)];
    v += load4f(bias + n);
    v += load4f(pos + (size_t)row * D + n);
    store4(out + ((size_t)b * (L + 1) + row) * D + n, v);
  }
};

// decoder_pred + drop cls + unpatchify ("nhwpqc->nchpwq", MCM.py:524-546, 683-686, 795-797)
struct EpiUnpatchify {
  float* img;
  const float* bias;
  int L, G, P, C, H, W;
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int b = m / L, p = m - b * L;
    const int hy = p / G, hx = p - hy * G;
    v += load4f(bias + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nn = n + j;
      const int q = nn / C, c = nn - q * C;
      const int py = q / P, px = q - py * P;
      img[(((size_t)b * C + c) * H + hy * P + py) * W + hx * P + px] = v[j];
    }
  }
};

// conv + PixelShuffle(2) (compressai subpel_conv3x3, r=2): out channel co = c*4 + i*2 + j goes to
// pixel (2y+i, 2x+j), channel c of the NHWC output.
template <int ACT> struct EpiPixelShuffle2 {
  float* out;
  const float* bias;
  int H, W, ldo;  // H, W: conv (input) resolution; ldo: output channel stride (= Cout/4 usually)
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int hw = H * W;
    const int b = m / hw, rem = m - b * hw;
    const int y = rem / W, x = rem - y * W;
    v += load4f(bias + n);
    const int c = n >> 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o = v[j];
      if (ACT == TMAE_ACT_GELU) o = gelu_erf(o);
      const int oy = 2 * y + (j >> 1), ox = 2 * x + (j & 1);
      out[(((size_t)b * 2 * H + oy) * 2 * W + ox) * ldo + c] = o;
    }
  }
};

// Fused scale conv epilogue: sigma = acc + bias, then compressai GaussianConditional likelihood
// (LowerBound(0.11) on the scale, erfc CDF, LowerBound(1e-9) on the likelihood; MCM.py:767-776)
// and y_hat = round(y - mu) + mu (quantize_ste forward value, MCM.py:776).
struct EpiGaussian {
  const float* y;       // NHWC latent, channel stride ldy, this slice at channel yoff
  const float* mu;      // NHWC slice means, channel stride ldmu
  const float* noise;   // optional NCHW [n][Mtot][H][W] uniform(-0.5, 0.5) (training)
  float* lik;           // NCHW [n][Mtot][H][W]
  float* yhat;          // NHWC support slot, channel stride ldh
  const float* bias;
  int ldy, yoff, ldmu, ldh, Mtot, HW;
  __device__ void operator()(int m, int n, f32x4 v) const {
    v += load4f(bias + n);
    const f32x4 yv = load4f(y + (size_t)m * ldy + yoff + n);
    const f32x4 mv = load4f(mu + (size_t)m * ldmu + n);
    const int b = m / HW, pix = m - b * HW;
    f32x4 yh;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t nchw = ((size_t)b * Mtot + yoff + n + j) * HW + pix;
      const float q = rintf(yv[j] - mv[j]) + mv[j];
      const float xt = noise ? yv[j] + noise[nchw] : q;
      const float s = fmaxf(v[j], 0.11f);
      const float val = fabsf(xt - mv[j]);
      const float c = -0.70710678118654752440f;
      const float up = 0.5f * erfcf(c * ((0.5f - val) / s));
      const float lo = 0.5f * erfcf(c * ((-0.5f - val) / s));
      lik[nchw] = fmaxf(up - lo, 1e-9f);
      yh[j] = q;
    }
    store4(yhat + (size_t)m * ldh + n, yh);
  }
};

// Fused LRP epilogue (MCM.py:779-784): y_hat += 0.5 * tanh(acc + bias); the pre-LRP y_hat is read
// from `src`, the result written to up to two destinations (full y_hat, support slot).
struct EpiLRP {
  const float* src;
  int lds;
  float* dst1;
  int ld1;
  float* dst2;  // optional
  int ld2;
  const float* bias;
  __device__ void operator()(int m, int n, f32x4 v) const {
    v += load4f(bias + n);
    f32x4 o = load4f(src + (size_t)m * lds + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = o[j] + 0.5f * tanhf(v[j]);
    store4(dst1 + (size_t)m * ld1 + n, o);
    if (dst2) store4(dst2 + (size_t)m * ld2 + n, o);
  }
};

// ------------------------------------------------------------------ the kernel
template <typename T, int BN, int BM, int WGN, class WL, class XL, class EPI>
__global__ void __launch_bounds__(256, 2)
gemm_kernel(const WL wl, const XL xl, const EPI epi, int M, int N, int K) {
  constexpr int EPC = Elt<T>::EPC;
  constexpr int BK = 8 * EPC;
  constexpr int WGM = 4 / WGN;
  constexpr int WN = BN / WGN, WM = BM / WGM;
  constexpr int TN = WN / 16, TM = WM / 16;
  constexpr int WCH = BN / 32, XCH = BM / 32;
  constexpr int ROWS = BN + BM;
  static_assert(TN >= 1 && TM >= 1 && WCH >= 1 && XCH >= 1, "bad tile");

  __shared__ uint4 lds[2 * ROWS * 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  const int ntn = (N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = bid % ntn, tm = bid / ntn;
  const int n0 = tn * BN, m0 = tm * BM;
  const int ch = tid & 7, r0 = tid >> 3;

  typename WL::Row wrow[WCH];
  typename XL::Row xrow[XCH];
#pragma unroll
  for (int p = 0; p < WCH; ++p) wrow[p] = wl.row(n0 + r0 + 32 * p);
#pragma unroll
  for (int p = 0; p < XCH; ++p) xrow[p] = xl.row(m0 + r0 + 32 * p);

  uint4 wreg[WCH], xreg[XCH];
  auto gload = [&](int kt) {
    const auto wc = wl.col(kt * 8 + ch);
    const auto xc = xl.col(kt * 8 + ch);
#pragma unroll
    for (int p = 0; p < WCH; ++p) wreg[p] = wl.load(wrow[p], wc);
#pragma unroll
    for (int p = 0; p < XCH; ++p) xreg[p] = xl.load(xrow[p], xc);
  };
  auto swrite = [&](int buf) {
    uint4* base = lds + buf * ROWS * 8;
#pragma unroll
    for (int p = 0; p < WCH; ++p) {
      const int r = r0 + 32 * p;
      base[r * 8 + (ch ^ ((r >> 1) & 7))] = wreg[p];
    }
#pragma unroll
    for (int p = 0; p < XCH; ++p) {
      const int r = r0 + 32 * p;
      base[(BN + r) * 8 + (ch ^ ((r >> 1) & 7))] = xreg[p];
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    const uint4* base = lds + (kt & 1) * ROWS * 8;
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 a[TN], b[TM];
        const int c = 4 * s + fq;
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int r = wn * WN + 16 * i + fr;
          uint4 u = base[r * 8 + (c ^ ((r >> 1) & 7))];
          a[i] = *reinterpret_cast<bf16x8*>(&u);
        }
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int r = wm * WM + 16 * j + fr;
          uint4 u = base[(BN + r) * 8 + (c ^ ((r >> 1) & 7))];
          b[j] = *reinterpret_cast<bf16x8*>(&u);
        }
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    } else {
      const float* fb = reinterpret_cast<const float*>(base);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float a[TN], b[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int r = wn * WN + 16 * i + fr;
          a[i] = fb[(r * 8 + (q ^ ((r >> 1) & 7))) * 4 + fq];
        }
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const int r = wm * WM + 16 * j + fr;
          b[j] = fb[((BN + r) * 8 + (q ^ ((r >> 1) & 7))) * 4 + fq];
        }
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) swrite((kt + 1) & 1);
    __syncthreads();
  }

#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn * WN + 16 * i + 4 * fq;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + 16 * j + fr;
      if (m < M && n < N) epi(m, n, acc[i][j]);
    }
  }
}

// ------------------------------------------------------------------ launch helpers
template <typename T, int BN, int BM, int WGN, class WL, class XL, class EPI>
static int launch_tile(const char* name, const WL& wl, const XL& xl, const EPI& epi, int M, int N, int K,
                       hipStream_t st) {
  const int grid = ceil_div(N, BN) * ceil_div(M, BM);
  if (grid == 0) return TMAE_OK;
  hipLaunchKernelGGL((gemm_kernel<T, BN, BM, WGN, WL, XL, EPI>), dim3(grid), dim3(256), 0, st, wl, xl, epi, M, N,
                     K);
  TMAE_LAUNCH_CHECK(name);
}

// Tile choice by output width N (weight rows): 128x128 for wide layers, narrower weight tiles for
// the 32..224-channel slice-transform convs so little MFMA work is spent on padding.
template <typename T, class XL, class EPI>
static int launch_gemm(const char* name, const T* w, int N, int K, const XL& xl, const EPI& epi, int M,
                       hipStream_t st) {
  DenseRows<T, T> wl{w, K, N, K, 1 << 30, 0, 0};
  if (N >= 256 && (N % 128 == 0 || N >= 512)) return launch_tile<T, 128, 128, 2>(name, wl, xl, epi, M, N, K, st);
  if (N > 96) return launch_tile<T, 64, 128, 1>(name, wl, xl, epi, M, N, K, st);
  return launch_tile<T, 32, 128, 1>(name, wl, xl, epi, M, N, K, st);
}

template <typename T> static int check_k(int K) { return (K % Elt<T>::EPC) == 0; }

// ------------------------------------------------------------------ C ABI
template <typename T>
static int linear_t(const void* x, int x_f32, int ldx, int G, int Gs, int off, const void* w, const float* bias,
                    void* y, int y_f32, int ldy, int M, int N, int K, int act, hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(K) && N % 4 == 0, "tmae_linear_fwd: K=%d must be a multiple of %d and N=%d of 4", K,
               Elt<T>::EPC, N);
  TMAE_REQUIRE(G > 0, "tmae_linear_fwd: row_group must be > 0");
  const T* W = (const T*)w;
#define TMAE_LIN_EPI(XL_)                                                                                     \
  do {                                                                                                        \
    if (y_f32) {                                                                                              \
      if (act == TMAE_ACT_GELU) return launch_gemm<T>("tmae_linear_fwd", W, N, K, XL_, EpiStore<float, 1>{(float*)y, ldy, bias}, M, st); \
      return launch_gemm<T>("tmae_linear_fwd", W, N, K, XL_, EpiStore<float, 0>{(float*)y, ldy, bias}, M, st);          \
    } else {                                                                                                  \
      if (act == TMAE_ACT_GELU) return launch_gemm<T>("tmae_linear_fwd", W, N, K, XL_, EpiStore<T, 1>{(T*)y, ldy, bias}, M, st); \
      return launch_gemm<T>("tmae_linear_fwd", W, N, K, XL_, EpiStore<T, 0>{(T*)y, ldy, bias}, M, st);                  \
    }                                                                                                         \
  } while (0)
  if (x_f32) {
    DenseRows<T, float> xl{(const float*)x, ldx, M, K, G, Gs, off};
    TMAE_LIN_EPI(xl);
  } else {
    DenseRows<T, T> xl{(const T*)x, ldx, M, K, G, Gs, off};
    TMAE_LIN_EPI(xl);
  }
#undef TMAE_LIN_EPI
}

extern "C" int tmae_linear_fwd(const void* x, int x_f32, int ldx, int row_group, int group_stride, int row_offset,
                               const void* w, const float* bias, void* y, int y_f32, int ldy, int M, int N, int K,
                               int act, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return linear_t<bf16>(x, x_f32, ldx, row_group, group_stride, row_offset, w, bias, y, y_f32, ldy, M, N, K, act,
                          (hipStream_t)stream);
  return linear_t<float>(x, 1, ldx, row_group, group_stride, row_offset, w, bias, y, 1, ldy, M, N, K, act,
                         (hipStream_t)stream);
}

template <typename T>
static int resid_t(const void* x, int ldx, const void* w, const float* bias, float* r, int ldr, int M, int N, int K,
                   hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(K) && N % 4 == 0, "tmae_linear_residual_fwd: bad K=%d / N=%d", K, N);
  DenseRows<T, T> xl{(const T*)x, ldx, M, K, 1 << 30, 0, 0};
  return launch_gemm<T>("tmae_linear_residual_fwd", (const T*)w, N, K, xl, EpiResidual{r, ldr, bias}, M, st);
}

extern "C" int tmae_linear_residual_fwd(const void* x, int ldx, const void* w, const float* bias, float* resid,
                                        int ldr, int M, int N, int K, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return resid_t<bf16>(x, ldx, w, bias, resid, ldr, M, N, K, (hipStream_t)stream);
  return resid_t<float>(x, ldx, w, bias, resid, ldr, M, N, K, (hipStream_t)stream);
}

template <typename T>
static int patch_t(const float* imgs, const int64_t* ids, const void* w, const float* bias, const float* pos,
                   float* tok, int n, int C, int H, int W, int P, int D, int L, int keep, hipStream_t st) {
  const int G = W / P;
  TMAE_REQUIRE(H == W && H % P == 0 && G * G == L, "tmae_patch_embed_fwd: image %dx%d, patch %d, L=%d mismatch", H,
               W, P, L);
  TMAE_REQUIRE(P % Elt<T>::EPC == 0 && D % 4 == 0, "tmae_patch_embed_fwd: patch %d / dim %d unsupported", P, D);
  const int K = C * P * P;
  PatchRows<T> xl{imgs, ids, L, keep, C, H, W, P, G, n * keep, K};
  return launch_gemm<T>("tmae_patch_embed_fwd", (const T*)w, D, K, xl, EpiPatchEmbed{tok, bias, pos, ids, L, keep, D},
                        n * keep, st);
}

extern "C" int tmae_patch_embed_fwd(const float* imgs, const int64_t* ids_shuffle, const void* w, const float* bias,
                                    const float* pos, float* tokens, int n, int C, int H, int W, int patch, int D,
                                    int L, int keep, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return patch_t<bf16>(imgs, ids_shuffle, w, bias, pos, tokens, n, C, H, W, patch, D, L, keep, (hipStream_t)stream);
  return patch_t<float>(imgs, ids_shuffle, w, bias, pos, tokens, n, C, H, W, patch, D, L, keep, (hipStream_t)stream);
}

template <typename T>
static int dec_embed_t(const void* x, int x_f32, const void* w, const float* bias, const float* pos,
                       const int64_t* ids, float* out, int n, int ntok, int L, int Din, int D, hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(Din) && D % 4 == 0, "tmae_decoder_embed_fwd: bad dims %d -> %d", Din, D);
  TMAE_REQUIRE(ntok >= 1 && ntok <= L + 1, "tmae_decoder_embed_fwd: ntok=%d, L=%d", ntok, L);
  EpiDecoderEmbed epi{out, bias, pos, ids, L, ntok, D};
  if (x_f32) {
    DenseRows<T, float> xl{(const float*)x, Din, n * ntok, Din, 1 << 30, 0, 0};
    return launch_gemm<T>("tmae_decoder_embed_fwd", (const T*)w, D, Din, xl, epi, n * ntok, st);
  }
  DenseRows<T, T> xl{(const T*)x, Din, n * ntok, Din, 1 << 30, 0, 0};
  return launch_gemm<T>("tmae_decoder_embed_fwd", (const T*)w, D, Din, xl, epi, n * ntok, st);
}

extern "C" int tmae_decoder_embed_fwd(const void* x, int x_f32, const void* w, const float* bias, const float* pos,
                                      const int64_t* ids_shuffle, float* out, int n, int ntok, int L, int Din, int D,
                                      int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return dec_embed_t<bf16>(x, x_f32, w, bias, pos, ids_shuffle, out, n, ntok, L, Din, D, (hipStream_t)stream);
  return dec_embed_t<float>(x, 1, w, bias, pos, ids_shuffle, out, n, ntok, L, Din, D, (hipStream_t)stream);
}

template <typename T>
static int dec_pred_t(const void* x, const void* w, const float* bias, float* imgs, int n, int L, int Din, int C,
                      int H, int W, int P, hipStream_t st) {
  const int G = W / P;
  const int N = P * P * C;
  TMAE_REQUIRE(H == W && G * G == L && check_k<T>(Din) && N % 4 == 0, "tmae_decoder_pred_fwd: bad geometry");
  DenseRows<T, T> xl{(const T*)x, Din, n * L, Din, 1 << 30, 0, 0};
  return launch_gemm<T>("tmae_decoder_pred_fwd", (const T*)w, N, Din, xl, EpiUnpatchify{imgs, bias, L, G, P, C, H, W},
                        n * L, st);
}

extern "C" int tmae_decoder_pred_fwd(const void* x, const void* w, const float* bias, float* imgs, int n, int L,
                                     int Din, int C, int H, int W, int patch, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return dec_pred_t<bf16>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
  return dec_pred_t<float>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
}

// ---- 3x3 convs
template <typename T>
static ConvRows<T> make_conv(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H, int W,
                             int stride) {
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  const int Cin = c1 + c2;
  ConvRows<T> xl;
  xl.x1 = x1; xl.x2 = x2; xl.c1 = c1; xl.ld1 = ld1; xl.ld2 = ld2; xl.Cin = Cin;
  xl.H = H; xl.W = W; xl.Ho = Ho; xl.Wo = Wo; xl.stride = stride; xl.rows = n * Ho * Wo; xl.K = 9 * Cin;
  xl.inv_cin = 1.0f / (float)Cin;
  return xl;
}

template <typename T>
static int conv_check(int c1, int ld1, int c2, int ld2, int cout) {
  const int e = Elt<T>::EPC;
  TMAE_REQUIRE(c1 % e == 0 && c2 % e == 0 && ld1 % 4 == 0 && (c2 == 0 || ld2 % 4 == 0) && cout % 4 == 0,
               "conv3x3: channel counts (%d + %d -> %d) must be multiples of %d", c1, c2, cout, e);
  return TMAE_OK;
}

template <typename T>
static int conv_t(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H, int W, int stride,
                  const void* w, const float* bias, float* y, int ldy, int cout, int act, int pshuf, hipStream_t st) {
  if (int e = conv_check<T>(c1, ld1, c2, ld2, cout)) return e;
  ConvRows<T> xl = make_conv<T>(x1, c1, ld1, x2, c2, ld2, n, H, W, stride);
  const int M = xl.rows, K = xl.K;
  const T* Wt = (const T*)w;
  if (pshuf) {
    TMAE_REQUIRE(stride == 1, "conv3x3: pixel shuffle needs stride 1");
    if (act == TMAE_ACT_GELU)
      return launch_gemm<T>("tmae_conv3x3_fwd", Wt, cout, K, xl, EpiPixelShuffle2<1>{y, bias, H, W, ldy}, M, st);
    return launch_gemm<T>("tmae_conv3x3_fwd", Wt, cout, K, xl, EpiPixelShuffle2<0>{y, bias, H, W, ldy}, M, st);
  }
  if (act == TMAE_ACT_GELU)
    return launch_gemm<T>("tmae_conv3x3_fwd", Wt, cout, K, xl, EpiStore<float, 1>{y, ldy, bias}, M, st);
  return launch_gemm<T>("tmae_conv3x3_fwd", Wt, cout, K, xl, EpiStore<float, 0>{y, ldy, bias}, M, st);
}

extern "C" int tmae_conv3x3_fwd(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H,
                                int W, int stride, const void* w, const float* bias, float* y, int ldy, int cout,
                                int act, int pixel_shuffle, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return conv_t<bf16>(x1, c1, ld1, x2, c2, ld2, n, H, W, stride, w, bias, y, ldy, cout, act, pixel_shuffle,
                        (hipStream_t)stream);
  return conv_t<float>(x1, c1, ld1, x2, c2, ld2, n, H, W, stride, w, bias, y, ldy, cout, act, pixel_shuffle,
                       (hipStream_t)stream);
}

template <typename T>
static int conv_gc_t(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H, int W,
                     const void* w, const float* bias, int cout, const float* y, int ldy, int yoff, const float* mu,
                     int ldmu, const float* noise, float* lik, int Mtot, float* yhat, int ldh, hipStream_t st) {
  if (int e = conv_check<T>(c1, ld1, c2, ld2, cout)) return e;
  ConvRows<T> xl = make_conv<T>(x1, c1, ld1, x2, c2, ld2, n, H, W, 1);
  EpiGaussian epi{y, mu, noise, lik, yhat, bias, ldy, yoff, ldmu, ldh, Mtot, H * W};
  return launch_gemm<T>("tmae_conv3x3_gaussian_fwd", (const T*)w, cout, xl.K, xl, epi, xl.rows, st);
}

extern "C" int tmae_conv3x3_gaussian_fwd(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n,
                                         int H, int W, const void* w, const float* bias, int cout, const float* y,
                                         int ldy, int yoff, const float* mu, int ldmu, const float* noise, float* lik,
                                         int Mtot, float* yhat, int ldh, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return conv_gc_t<bf16>(x1, c1, ld1, x2, c2, ld2, n, H, W, w, bias, cout, y, ldy, yoff, mu, ldmu, noise, lik, Mtot,
                           yhat, ldh, (hipStream_t)stream);
  return conv_gc_t<float>(x1, c1, ld1, x2, c2, ld2, n, H, W, w, bias, cout, y, ldy, yoff, mu, ldmu, noise, lik, Mtot,
                          yhat, ldh, (hipStream_t)stream);
}

template <typename T>
static int conv_lrp_t(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H, int W,
                      const void* w, const float* bias, int cout, const float* src, int lds, float* dst1, int ld1o,
                      float* dst2, int ld2o, hipStream_t st) {
  if (int e = conv_check<T>(c1, ld1, c2, ld2, cout)) return e;
  ConvRows<T> xl = make_conv<T>(x1, c1, ld1, x2, c2, ld2, n, H, W, 1);
  EpiLRP epi{src, lds, dst1, ld1o, dst2, ld2o, bias};
  return launch_gemm<T>("tmae_conv3x3_lrp_fwd", (const T*)w, cout, xl.K, xl, epi, xl.rows, st);
}

extern "C" int tmae_conv3x3_lrp_fwd(const float* x1, int c1, int ld1, const float* x2, int c2, int ld2, int n, int H,
                                    int W, const void* w, const float* bias, int cout, const float* src, int ld_src,
                                    float* dst1, int ld_dst1, float* dst2, int ld_dst2, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return conv_lrp_t<bf16>(x1, c1, ld1, x2, c2, ld2, n, H, W, w, bias, cout, src, ld_src, dst1, ld_dst1, dst2,
                            ld_dst2, (hipStream_t)stream);
  return conv_lrp_t<float>(x1, c1, ld1, x2, c2, ld2, n, H, W, w, bias, cout, src, ld_src, dst1, ld_dst1, dst2, ld_dst2,
                           (hipStream_t)stream);
}
