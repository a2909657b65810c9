// LIC 3x3 convolutions (h_a, h_s, cc_transform_mean/scale, lrp_transform; MCM.py:115-293) as
// implicit GEMMs on the MFMA core, batched over independent problems (mean/scale chains of one
// slice; slices 6..11 whose support is fixed), plus the Gaussian-conditional slice kernel.
#include "conv_halo.h"
#include "gemm_core.h"

// conv + PixelShuffle(2) (compressai subpel_conv3x3, r=2): conv channel co = c*4 + i*2 + j goes to
// pixel (2y+i, 2x+j), channel c of the NHWC output.
template <typename OT, int ACT> struct EpiPixelShuffle2 {
  OT* out;
  const float* bias;
  int H, W, ldo;
  BStride so, sb;
  OT* pre = nullptr;  // optional pre-activation copy, same (shuffled) layout as out
  BStride sp = {0, 0};
  __device__ void batch(int b1, int b2) {
    out += so.at(b1, b2);
    bias += sb.at(b1, b2);
    if (pre) pre += sp.at(b1, b2);
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int hw = H * W;
    const int b = m / hw, rem = m - b * hw;
    const int y = rem / W, x = rem - y * W;
    v += load4f(bias + n);
    const int c = n >> 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o = v[j];
      const int oy = 2 * y + (j >> 1), ox = 2 * x + (j & 1);
      const size_t at = (((size_t)b * 2 * H + oy) * 2 * W + ox) * ldo + c;
      if (pre) pre[at] = to_out<OT>(o);
      if (ACT == TMAE_ACT_GELU) o = gelu_for<OT>(o);
      out[at] = to_out<OT>(o);
    }
  }
  f32x4 pb0, pb1;  // this lane's bias columns (epilogue_lds prefetch hook)
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  // 8 columns = output channels c, c+1 of the 4 sub-pixels: four 2-channel stores
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const {
    const int hw = H * W;
    const int b = m / hw, rem = m - b * hw;
    const int y = rem / W, x = rem - y * W;
    lo += pb0; hi += pb1;
    const int c = n >> 2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float o0 = lo[j], o1 = hi[j];
      const int oy = 2 * y + (j >> 1), ox = 2 * x + (j & 1);
      const size_t at = (((size_t)b * 2 * H + oy) * 2 * W + ox) * ldo + c;
      if (pre) { pre[at] = to_out<OT>(o0); pre[at + 1] = to_out<OT>(o1); }
      if (ACT == TMAE_ACT_GELU) { o0 = gelu_for<OT>(o0); o1 = gelu_for<OT>(o1); }
      OT* p = out + at;
      p[0] = to_out<OT>(o0);
      p[1] = to_out<OT>(o1);
    }
  }
};

// last lrp_transform conv: y_hat = y_hat_pre + 0.5 * tanh(acc + bias)  (MCM.py:779-784)
template <typename OT> struct EpiLRP {
  const float* src;
  int lds;
  OT* out;
  int ldo;
  OT* out2;  // optional
  int ldo2;
  const float* bias;
  BStride ssrc, so, so2, sb;
  float* pre = nullptr;  // optional pre-tanh value (training: tanh' in the backward)
  int ldp = 0;
  BStride sp = {0, 0};
  __device__ void batch(int b1, int b2) {
    src += ssrc.at(b1, b2);
    out += so.at(b1, b2);
    if (out2) out2 += so2.at(b1, b2);
    bias += sb.at(b1, b2);
    if (pre) pre += sp.at(b1, b2);
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    v += load4f(bias + n);
    if (pre) store4(pre + (size_t)m * ldp + n, v);
    f32x4 o = load4f(src + (size_t)m * lds + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = o[j] + 0.5f * tanhf(v[j]);
    store4(out + (size_t)m * ldo + n, o);
    if (out2) store4(out2 + (size_t)m * ldo2 + n, o);
  }
  // epilogue_lds hooks: bias once per lane, the y_hat_pre rows one block ahead
  f32x4 pb0, pb1;
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  struct Pre { f32x4 o0, o1; };
  __device__ Pre fetch(int m, int n) const {
    Pre p;
    load8f(src + (size_t)m * lds + n, p.o0, p.o1);
    return p;
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi, const Pre& p) const {
    f32x4 o0 = p.o0, o1 = p.o1;
    lo += pb0; hi += pb1;
    if (pre) store8(pre + (size_t)m * ldp + n, lo, hi);
#pragma unroll
    for (int j = 0; j < 4; ++j) { o0[j] += 0.5f * tanhf(lo[j]); o1[j] += 0.5f * tanhf(hi[j]); }
    store8(out + (size_t)m * ldo + n, o0, o1);
    if (out2) store8(out2 + (size_t)m * ldo2 + n, o0, o1);
  }};

// bf16 stride-1 12x12 convs go to the halo-staged kernel (conv_halo.h); everything else (f32 parity
// path, strided / 6x6 / 3x3 maps, wide N) to the implicit GEMM
template <typename T, class XS, class EPI>
static int conv_go(const char* nm, const tmae_conv_args& a, const T* W, int N, int K, int M, const XS& xs,
                   const EPI& epi, hipStream_t st) {
  if constexpr (sizeof(T) == 2) {
    if (conv_halo_ok(a.H, a.W, a.stride, N, a.nb1 * a.nb2)) {
      const HaloSrc hs{(const bf16*)a.x1, (const bf16*)a.x2, a.c1, a.ld1, a.ld2, a.c1 + a.c2,
                       BStride{a.x1_s1, a.x1_s2}, BStride{a.x2_s1, a.x2_s2}};
      return launch_conv_halo(nm, W, BStride{a.w_s1, a.w_s2}, hs, epi, N, a.n, a.nb1, a.nb2, st);
    }
  }
  if constexpr (sizeof(T) == 2 && std::is_same<XS, ConvSrc<T>>::value) {
    if (xs.Cin >= 128) {  // the K iterator source (gemm_core.h ConvSrcIt): wide inputs only
      ConvSrcIt<T> xi;
      static_cast<ConvSrc<T>&>(xi) = xs;
      return launch_gemm<true, T>(nm, W, a.w_s1, a.w_s2, N, K, xi, epi, M, a.nb1, a.nb2, st);
    }
  }
  return launch_gemm<true, T>(nm, W, a.w_s1, a.w_s2, N, K, xs, epi, M, a.nb1, a.nb2, st);
}

template <typename T>
static int conv_t(const tmae_conv_args& a, hipStream_t st) {
  const int e = Elt<T>::EPC;
  TMAE_REQUIRE(a.c1 % e == 0 && a.c2 % e == 0 && a.ld1 % e == 0 && (a.c2 == 0 || a.ld2 % e == 0) && a.cout % 4 == 0,
               "tmae_conv3x3: channel counts (%d + %d -> %d) must be multiples of %d", a.c1, a.c2, a.cout, e);
  TMAE_REQUIRE(a.stride == 1 || a.stride == 2, "tmae_conv3x3: stride %d", a.stride);
  TMAE_REQUIRE(!(a.pixel_shuffle && a.lrp_src), "tmae_conv3x3: pixel_shuffle and lrp are exclusive");
  TMAE_REQUIRE(a.act != TMAE_ACT_RELU || (!a.pixel_shuffle && !a.lrp_src), "tmae_conv3x3: ReLU on a plain store only");
  TMAE_REQUIRE(a.nb1 >= 1 && a.nb2 >= 1, "tmae_conv3x3: batch %d x %d", a.nb1, a.nb2);
  ConvSrc<T> xs;
  xs.x1 = (const T*)a.x1; xs.x2 = (const T*)a.x2; xs.c1 = a.c1; xs.ld1 = a.ld1; xs.ld2 = a.ld2;
  xs.Cin = a.c1 + a.c2; xs.H = a.H; xs.W = a.W;
  xs.Ho = (a.H + 2 - 3) / a.stride + 1; xs.Wo = (a.W + 2 - 3) / a.stride + 1; xs.stride = a.stride;
  xs.rows = a.n * xs.Ho * xs.Wo; xs.K = 9 * xs.Cin; xs.inv_cin = xs.Cin ? 1.0f / (float)xs.Cin : 0.0f;
  xs.bs1 = BStride{a.x1_s1, a.x1_s2}; xs.bs2 = BStride{a.x2_s1, a.x2_s2};
  const int M = xs.rows, K = xs.K, N = a.cout;
  const T* W = (const T*)a.w;
  const char* nm = "tmae_conv3x3";
#define TMAE_GO(EPI) return conv_go<T>(nm, a, W, N, K, M, xs, EPI, st)
  if (a.pixel_shuffle) {
    TMAE_REQUIRE(a.stride == 1, "tmae_conv3x3: pixel shuffle needs stride 1");
    if (a.y_f32) {
      EpiPixelShuffle2<float, 1> g{(float*)a.y, a.bias, a.H, a.W, a.ldy, {a.y_s1, a.y_s2}, {a.b_s1, a.b_s2},
                                   (float*)a.pre, {a.pre_s1, a.pre_s2}};
      EpiPixelShuffle2<float, 0> l{(float*)a.y, a.bias, a.H, a.W, a.ldy, {a.y_s1, a.y_s2}, {a.b_s1, a.b_s2},
                                   (float*)a.pre, {a.pre_s1, a.pre_s2}};
      if (a.act == TMAE_ACT_GELU) TMAE_GO(g);
      TMAE_GO(l);
    }
    EpiPixelShuffle2<T, 1> g{(T*)a.y, a.bias, a.H, a.W, a.ldy, {a.y_s1, a.y_s2}, {a.b_s1, a.b_s2},
                             (T*)a.pre, {a.pre_s1, a.pre_s2}};
    EpiPixelShuffle2<T, 0> l{(T*)a.y, a.bias, a.H, a.W, a.ldy, {a.y_s1, a.y_s2}, {a.b_s1, a.b_s2},
                             (T*)a.pre, {a.pre_s1, a.pre_s2}};
    if (a.act == TMAE_ACT_GELU) TMAE_GO(g);
    TMAE_GO(l);
  }
  if (a.lrp_src) {
    TMAE_REQUIRE(!a.y_f32 || sizeof(T) == 4, "tmae_conv3x3: lrp output must be in the operand dtype");
    EpiLRP<T> r{a.lrp_src, a.ld_src, (T*)a.y, a.ldy, (T*)a.y2, a.ldy2, a.bias, {a.src_s1, a.src_s2},
                {a.y_s1, a.y_s2}, {a.y2_s1, a.y2_s2}, {a.b_s1, a.b_s2}, (float*)a.pre, a.ldp, {a.pre_s1, a.pre_s2}};
    TMAE_GO(r);
  }
  if (a.act == TMAE_ACT_RELU) {  // VGG16 (loss/vgg.py): plain conv + ReLU, no addend / copies
    TMAE_REQUIRE(!a.addend && !a.pre, "tmae_conv3x3: ReLU supports plain stores (+ an f32 copy) only");
    if (a.y_f32) {
      auto r = make_store<float, TMAE_ACT_RELU>((float*)a.y, a.ldy, a.bias);
      r.so = BStride{a.y_s1, a.y_s2};
      r.sb = BStride{a.b_s1, a.b_s2};
      return launch_gemm<true, T>(nm, W, a.w_s1, a.w_s2, N, K, xs, r, M, a.nb1, a.nb2, st);
    }
    auto r = make_store<T, TMAE_ACT_RELU>((T*)a.y, a.ldy, a.bias);
    r.so = BStride{a.y_s1, a.y_s2};
    r.sb = BStride{a.b_s1, a.b_s2};
    r.out32 = a.y32;
    r.ld32 = a.ld32;
    r.s32 = BStride{a.y32_s1, a.y32_s2};
    return launch_gemm<true, T>(nm, W, a.w_s1, a.w_s2, N, K, xs, r, M, a.nb1, a.nb2, st);
  }
  if (a.y_f32) {
    auto g = make_store<float, 1>((float*)a.y, a.ldy, a.bias);
    auto l = make_store<float, 0>((float*)a.y, a.ldy, a.bias);
    g.so = l.so = BStride{a.y_s1, a.y_s2};
    g.sb = l.sb = BStride{a.b_s1, a.b_s2};
    g.addend = l.addend = a.addend;
    g.ld_add = l.ld_add = a.ld_add;
    g.sa = l.sa = BStride{a.a_s1, a.a_s2};
    g.pre = l.pre = (float*)a.pre;
    g.ldp = l.ldp = a.ldp;
    g.sp = l.sp = BStride{a.pre_s1, a.pre_s2};
    if (a.act == TMAE_ACT_GELU) TMAE_GO(g);
    TMAE_GO(l);
  }
  auto g = make_store<T, 1>((T*)a.y, a.ldy, a.bias);
  auto l = make_store<T, 0>((T*)a.y, a.ldy, a.bias);
  g.so = l.so = BStride{a.y_s1, a.y_s2};
  g.sb = l.sb = BStride{a.b_s1, a.b_s2};
  g.addend = l.addend = a.addend;
  g.ld_add = l.ld_add = a.ld_add;
  g.sa = l.sa = BStride{a.a_s1, a.a_s2};
  g.out32 = l.out32 = a.y32;
  g.ld32 = l.ld32 = a.ld32;
  g.s32 = l.s32 = BStride{a.y32_s1, a.y32_s2};
  g.pre = l.pre = (T*)a.pre;
  g.ldp = l.ldp = a.ldp;
  g.sp = l.sp = BStride{a.pre_s1, a.pre_s2};
  if (a.act == TMAE_ACT_GELU) TMAE_GO(g);
  TMAE_GO(l);
#undef TMAE_GO
}

extern "C" int tmae_conv3x3(const tmae_conv_args* args, int dtype, void* stream) {
  TMAE_REQUIRE(args != nullptr, "tmae_conv3x3: args is NULL");
  if (dtype == TMAE_BF16) return conv_t<bf16>(*args, (hipStream_t)stream);
  TMAE_REQUIRE(args->y_f32 || args->lrp_src, "tmae_conv3x3: the f32 path writes f32 outputs");
  return conv_t<float>(*args, (hipStream_t)stream);
}

// ------------------------------------------------------------------ Gaussian conditional, per slice
// compressai GaussianConditional forward (LowerBound(0.11) on scales, erfc CDF, LowerBound(1e-9))
// for `nslices` consecutive slices of width sw, and y_hat = round(y - mu) + mu (quantize_ste forward
// value, MCM.py:767-776).  Element (pixel m, slice j, channel c) of the latent channel
// ch = yoff + j*sw + c; mu/sigma of slice j at mu[j*ms_stride + m*ld_ms + c].
template <typename YT, bool CODE>
__global__ void __launch_bounds__(256)
gc_slices_kernel(const float* __restrict__ y, int ldy, int yoff, const float* __restrict__ mu,
                 const float* __restrict__ sigma, long long ms_stride, int ld_ms, const float* __restrict__ noise,
                 float* __restrict__ lik, int Mtot, YT* __restrict__ yhat, int ld_yhat, float* __restrict__ yhat32,
                 int ld32, int n, int HW, int nslices, int sw, int total, int* __restrict__ sym,
                 int* __restrict__ idx, const float* __restrict__ scale_table, int nscale) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int per_pix = nslices * sw;
  const int m = i / per_pix, r = i - m * per_pix;
  const int j = r / sw, c = r - j * sw;
  const int ch = yoff + j * sw + c;
  const int b = m / HW, pix = m - b * HW;
  const float yv = y[(size_t)m * ldy + ch];
  const float mv = mu[j * ms_stride + (size_t)m * ld_ms + c];
  const float sv = sigma[j * ms_stride + (size_t)m * ld_ms + c];
  const size_t nchw = ((size_t)b * Mtot + ch) * HW + pix;
  const float qi = rintf(yv - mv);
  const float q = qi + mv;
  const float xt = noise ? yv + noise[nchw] : q;
  const float s = fmaxf(sv, 0.11f);
  const float val = fabsf(xt - mv);
  const float k = -0.70710678118654752440f;
  const float up = 0.5f * erfcf(k * ((0.5f - val) / s));
  const float lo = 0.5f * erfcf(k * ((-0.5f - val) / s));
  lik[nchw] = fmaxf(up - lo, 1e-9f);
  if (yhat) yhat[(size_t)m * ld_yhat + ch] = to_out<YT>(q);
  if (yhat32) yhat32[(size_t)m * ld32 + ch] = q;
  if constexpr (CODE) {
    // MCM.compress (MCM.py:867-872): symbols = round(y - mu) (quantize "symbols"), indexes =
    // GaussianConditional.build_indexes(sigma); reference order per slice = [N][sw][H][W], slice-major
    const size_t pos = (size_t)j * n * sw * HW + ((size_t)b * sw + c) * HW + pix;
    sym[pos] = (int)qi;
    int id = nscale - 1;
    for (int t = 0; t < nscale - 1; ++t) id -= (s <= scale_table[t]) ? 1 : 0;
    idx[pos] = id;
  }
}

// The same per element, one 1024-thread workgroup per (image, slice) over its HW x sw block (bench: 144 x 32; 256
// threads left 6 waves per CU and ran 48 vs 34 us per forward), so that BOTH
// layouts are written whole-line: y / mu / sigma are read and y_hat / y_hat f32 written in the NHWC order
// (channel fastest), then y, mu and the bounded scale go through LDS and the likelihood (NCHW), the training
// noise (NCHW) and the compress symbols / indexes ([slice][N][sw][H][W]) are read / written pixel fastest.
// The element kernel above wrote the NCHW likelihoods 4 B per lane at a 576-B stride, a line's 32 pixels from
// ~24 workgroups spread over the XCDs (PMC: 1.92x the algorithmic bytes, partial lines written back by
// several L2s).  Same arithmetic per element: bitwise the same outputs.
constexpr int GC_TILE_MAX = 4800;  // HW * (sw + 1) floats per LDS array (3 arrays, 57.6 KB)
template <typename YT, bool CODE>
__global__ void __launch_bounds__(1024)
gc_slices_tiled_kernel(const float* __restrict__ y, int ldy, int yoff, const float* __restrict__ mu,
                       const float* __restrict__ sigma, long long ms_stride, int ld_ms, const float* __restrict__ noise,
                       float* __restrict__ lik, int Mtot, YT* __restrict__ yhat, int ld_yhat, float* __restrict__ yhat32,
                       int ld32, int n, int HW, int nslices, int sw, int* __restrict__ sym, int* __restrict__ idx,
                       const float* __restrict__ scale_table, int nscale) {
  __shared__ float ys[GC_TILE_MAX], ms[GC_TILE_MAX], ss[GC_TILE_MAX];
  const int b = blockIdx.x / nslices, j = blockIdx.x - b * nslices;
  const int ld = sw + 1, tot = HW * sw;
  // phase 1: NHWC order
  for (int e = threadIdx.x; e < tot; e += 1024) {
    const int pix = e / sw, c = e - pix * sw;
    const int m = b * HW + pix, ch = yoff + j * sw + c;
    const float yv = y[(size_t)m * ldy + ch];
    const float mv = mu[j * ms_stride + (size_t)m * ld_ms + c];
    const float sv = sigma[j * ms_stride + (size_t)m * ld_ms + c];
    const float q = rintf(yv - mv) + mv;
    if (yhat) yhat[(size_t)m * ld_yhat + ch] = to_out<YT>(q);
    if (yhat32) yhat32[(size_t)m * ld32 + ch] = q;
    ys[pix * ld + c] = yv;
    ms[pix * ld + c] = mv;
    ss[pix * ld + c] = fmaxf(sv, 0.11f);
  }
  __syncthreads();
  // phase 2: NCHW order (pixel fastest)
  for (int e = threadIdx.x; e < tot; e += 1024) {
    const int c = e / HW, pix = e - c * HW;
    const int ch = yoff + j * sw + c;
    const float yv = ys[pix * ld + c], mv = ms[pix * ld + c], s = ss[pix * ld + c];
    const size_t nchw = ((size_t)b * Mtot + ch) * HW + pix;
    const float qi = rintf(yv - mv);
    const float q = qi + mv;
    const float xt = noise ? yv + noise[nchw] : q;
    const float val = fabsf(xt - mv);
    const float k = -0.70710678118654752440f;
    const float up = 0.5f * erfcf(k * ((0.5f - val) / s));
    const float lo = 0.5f * erfcf(k * ((-0.5f - val) / s));
    lik[nchw] = fmaxf(up - lo, 1e-9f);
    if constexpr (CODE) {
      const size_t pos = (size_t)j * n * sw * HW + ((size_t)b * sw + c) * HW + pix;
      sym[pos] = (int)qi;
      int id = nscale - 1;
      for (int t = 0; t < nscale - 1; ++t) id -= (s <= scale_table[t]) ? 1 : 0;
      idx[pos] = id;
    }
  }
}

template <bool CODE>
static int gc_slices_launch(const float* y, int ldy, int yoff, const float* mu, const float* sigma,
                            long long ms_stride, int ld_ms, const float* noise, float* lik, int Mtot, void* yhat,
                            int yhat_dtype, int ld_yhat, float* yhat32, int ld32, int n, int HW, int nslices, int sw,
                            int* sym, int* idx, const float* scale_table, int nscale, hipStream_t st) {
  const int total = n * HW * nslices * sw;
  if (total <= 0) return TMAE_OK;
  if (HW * (sw + 1) <= GC_TILE_MAX) {
    const dim3 tg(n * nslices);
    if (yhat_dtype == TMAE_BF16)
      hipLaunchKernelGGL((gc_slices_tiled_kernel<bf16, CODE>), tg, dim3(1024), 0, st, y, ldy, yoff, mu, sigma, ms_stride,
                         ld_ms, noise, lik, Mtot, (bf16*)yhat, ld_yhat, yhat32, ld32, n, HW, nslices, sw, sym, idx,
                         scale_table, nscale);
    else
      hipLaunchKernelGGL((gc_slices_tiled_kernel<float, CODE>), tg, dim3(1024), 0, st, y, ldy, yoff, mu, sigma,
                         ms_stride, ld_ms, noise, lik, Mtot, (float*)yhat, ld_yhat, yhat32, ld32, n, HW, nslices, sw,
                         sym, idx, scale_table, nscale);
    TMAE_LAUNCH_CHECK(CODE ? "tmae_gc_slices_code" : "tmae_gc_slices_fwd");
  }
  // maps past the LDS tile (HW * (sw + 1) > 4800 floats): one element per thread
  const dim3 grid(ceil_div(total, 256));
  if (yhat_dtype == TMAE_BF16)
    hipLaunchKernelGGL((gc_slices_kernel<bf16, CODE>), grid, dim3(256), 0, st, y, ldy, yoff, mu, sigma, ms_stride,
                       ld_ms, noise, lik, Mtot, (bf16*)yhat, ld_yhat, yhat32, ld32, n, HW, nslices, sw, total, sym, idx,
                       scale_table, nscale);
  else
    hipLaunchKernelGGL((gc_slices_kernel<float, CODE>), grid, dim3(256), 0, st, y, ldy, yoff, mu, sigma, ms_stride,
                       ld_ms, noise, lik, Mtot, (float*)yhat, ld_yhat, yhat32, ld32, n, HW, nslices, sw, total, sym,
                       idx, scale_table, nscale);
  TMAE_LAUNCH_CHECK(CODE ? "tmae_gc_slices_code" : "tmae_gc_slices_fwd");
}

extern "C" int tmae_gc_slices_fwd(const float* y, int ldy, int yoff, const float* mu, const float* sigma,
                                  long long ms_stride, int ld_ms, const float* noise, float* lik, int Mtot,
                                  void* yhat, int yhat_dtype, int ld_yhat, float* yhat32, int ld32, int n, int HW,
                                  int nslices, int sw, void* stream) {
  return gc_slices_launch<false>(y, ldy, yoff, mu, sigma, ms_stride, ld_ms, noise, lik, Mtot, yhat, yhat_dtype,
                                 ld_yhat, yhat32, ld32, n, HW, nslices, sw, nullptr, nullptr, nullptr, 0,
                                 (hipStream_t)stream);
}

extern "C" int tmae_gc_slices_code(const float* y, int ldy, int yoff, const float* mu, const float* sigma,
                                   long long ms_stride, int ld_ms, float* lik, int Mtot, void* yhat, int yhat_dtype,
                                   int ld_yhat, float* yhat32, int ld32, int n, int HW, int nslices, int sw,
                                   int* symbols, int* indexes, const float* scale_table, int nscale, void* stream) {
  TMAE_REQUIRE(symbols && indexes && scale_table && nscale >= 1, "tmae_gc_slices_code: symbols/indexes/scale_table required");
  return gc_slices_launch<true>(y, ldy, yoff, mu, sigma, ms_stride, ld_ms, nullptr, lik, Mtot, yhat, yhat_dtype,
                                ld_yhat, yhat32, ld32, n, HW, nslices, sw, symbols, indexes, scale_table, nscale,
                                (hipStream_t)stream);
}
