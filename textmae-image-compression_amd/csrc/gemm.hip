// Token-matrix GEMMs of the ViT encoder/decoder and the 1x1 LIC transforms, on the MFMA core
// (gemm_core.h).  Entry points and the reference computation each replaces: include/tmae.h.
#include <stdio.h>

#include "gemm_core.h"


// f32 rows converted to T on the way in (register-staged kernel only)
template <typename T> struct DenseSrcF32 {
  const float* p;
  int ld, rows, K, G, Gs, off;
  struct Row { const float* ptr; };
  __device__ void batch(int, int) {}
  __device__ Row row(int m) const {
    if (m >= rows) return {nullptr};
    return {p + (size_t)((m / G) * Gs + off + (m % G)) * ld};
  }
  __device__ uint4 load(const Row& r, int kt, int c) const {
    const int k = kt * 8 * Elt<T>::EPC + c * Elt<T>::EPC;
    if (!r.ptr || k >= K) return uint4{0, 0, 0, 0};
    return load_chunk_from_f32<T>(r.ptr + k);
  }
};

// residual stream update x += W·a + b (timm Block residual adds)
struct EpiResidual {
  float* out;
  int ldo;
  const float* bias;
  __device__ void batch(int, int) {}
  __device__ void operator()(int m, int n, f32x4 v) const {
    float* p = out + (size_t)m * ldo + n;
    if (bias) v += load4f(bias + n);
    store4(p, load4f(p) + v);
  }
  // epilogue_lds hooks (gemm_core.h): bias once per lane, the residual rows one block ahead
  f32x4 pb0, pb1;
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias && n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  struct Pre { f32x4 r0, r1; };
  __device__ Pre fetch(int m, int n) const {
    Pre p;
    load8f(out + (size_t)m * ldo + n, p.r0, p.r1);
    return p;
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi, const Pre& p) const {
    store8(out + (size_t)m * ldo + n, p.r0 + (lo + pb0), p.r1 + (hi + pb1));
  }};

// patch embed: token row b*(keep+1) + 1 + k  <-  acc + bias + pos[1 + p]   (MCM.py:615-626)
struct EpiPatchEmbed {
  float* tok;
  const float* bias;
  const float* pos;
  const int64_t* ids;
  int L, keep, D;
  __device__ void batch(int, int) {}
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int b = m / keep, k = m - b * keep;
    const int p = (int)ids[(size_t)b * L + k];
    v += load4f(bias + n);
    v += load4f(pos + (size_t)(1 + p) * D + n);
    store4(tok + ((size_t)b * (keep + 1) + 1 + k) * D + n, v);
  }
  f32x4 pb0, pb1;  // this lane's bias columns (epilogue_lds prefetch hook)
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const {
    const int b = m / keep, k = m - b * keep;
    const int p = (int)ids[(size_t)b * L + k];
    f32x4 p0, p1;
    load8f(pos + (size_t)(1 + p) * D + n, p0, p1);
    store8(tok + ((size_t)b * (keep + 1) + 1 + k) * D + n, lo + pb0 + p0, hi + pb1 + p1);
  }
};

// decoder embed + unshuffle (MCM.py:657-675; models_mae.py forward_decoder): token k of image b
// goes to decoder row 0 if k == 0, else 1 + ids_shuffle[b][k-1]; + decoder_pos_embed.
struct EpiDecoderEmbed {
  float* out;
  const float* bias;
  const float* pos;
  const int64_t* ids;
  int L, ntok, D;
  __device__ void batch(int, int) {}
  __device__ void operator()(int m, int n, f32x4 v) const {
    const int b = m / ntok, k = m - b * ntok;
    const int row = (k == 0) ? 0 : 1 + (int)ids[(size_t)b * L + (k - 1)];
    v += load4f(bias + n);
    v += load4f(pos + (size_t)row * D + n);
    store4(out + ((size_t)b * (L + 1) + row) * D + n, v);
  }
  f32x4 pb0, pb1;  // this lane's bias columns (epilogue_lds prefetch hook)
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const {
    const int b = m / ntok, k = m - b * ntok;
    const int row = (k == 0) ? 0 : 1 + (int)ids[(size_t)b * L + (k - 1)];
    f32x4 p0, p1;
    load8f(pos + (size_t)row * D + n, p0, p1);
    store8(out + ((size_t)b * (L + 1) + row) * D + n, lo + pb0 + p0, hi + pb1 + p1);
  }
};

// decoder_pred + drop cls + unpatchify ("nhwpqc->nchpwq", MCM.py:524-546, 683-686, 795-797)
struct EpiUnpatchify {
  float* img;
  const float* bias;
  int L, G, P, C, H, W;
  __device__ void batch(int, int) {}
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

// decoder_pred + unpatchify with channel-planar weight rows: row n = (c*P + py)*P + px (the reference's
// (py*P + px)*C + c, permuted once on the host). Eight consecutive columns are then eight consecutive
// pixels of one image row, so a lane's wide emit is two 16-B stores instead of eight 4-B stores spread
// over three channel planes.
struct EpiUnpatchifyCP {
  float* img;
  const float* bias;
  int L, G, P, C, H, W;
  __device__ void batch(int, int) {}
  __device__ float* pix(int m, int nn) const {
    const int b = m / L, p = m - b * L;
    const int hy = p / G, hx = p - hy * G;
    const int c = nn / (P * P), r = nn - c * P * P;
    const int py = r / P, px = r - py * P;
    return img + (((size_t)b * C + c) * H + hy * P + py) * W + hx * P + px;
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    v += load4f(bias + n);
#pragma unroll
    for (int j = 0; j < 4; ++j) *pix(m, n + j) = v[j];
  }
  f32x4 pb0, pb1;  // this lane's bias columns (epilogue_lds prefetch hook)
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  // n is a multiple of 8; with P % 8 == 0 (host-checked) the 8 columns share (c, py)
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const {
    float* o = pix(m, n);
    store4(o, lo + pb0);
    store4(o + 4, hi + pb1);
  }
};

// out = resid + W·a + b, out-of-place (training keeps the block input for the LayerNorm backward)
struct EpiResidualOut {
  const float* resid;
  float* out;
  int ld;
  const float* bias;
  __device__ void batch(int, int) {}
  __device__ void operator()(int m, int n, f32x4 v) const {
    if (bias) v += load4f(bias + n);
    store4(out + (size_t)m * ld + n, load4f(resid + (size_t)m * ld + n) + v);
  }
  f32x4 pb0, pb1;
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias && n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  struct Pre { f32x4 r0, r1; };
  __device__ Pre fetch(int m, int n) const {
    Pre p;
    load8f(resid + (size_t)m * ld + n, p.r0, p.r1);
    return p;
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi, const Pre& p) const {
    store8(out + (size_t)m * ld + n, p.r0 + (lo + pb0), p.r1 + (hi + pb1));
  }};

template <typename T> static int check_k(int K) { return (K % Elt<T>::EPC) == 0; }

// ------------------------------------------------------------------ linear
template <typename T, class XS, bool GLDS>
static int linear_epi(const T* W, int N, int K, const XS& xs, void* y, int y_f32, int ldy, float* y32, int ld32,
                      const float* bias, int M, int act, hipStream_t st, void* pre = nullptr, int ldp = 0) {
  const char* nm = "tmae_linear_fwd";
  if (y_f32) {
    auto e0 = make_store<float, 0>((float*)y, ldy, bias);
    auto e1 = make_store<float, 1>((float*)y, ldy, bias);
    e0.pre = e1.pre = (float*)pre;
    e0.ldp = e1.ldp = ldp;
    return act == TMAE_ACT_GELU ? launch_gemm<GLDS, T>(nm, W, 0, 0, N, K, xs, e1, M, 1, 1, st)
                                : launch_gemm<GLDS, T>(nm, W, 0, 0, N, K, xs, e0, M, 1, 1, st);
  }
  auto e0 = make_store<T, 0>((T*)y, ldy, bias);
  auto e1 = make_store<T, 1>((T*)y, ldy, bias);
  e0.out32 = e1.out32 = y32;
  e0.ld32 = e1.ld32 = ld32;
  e0.pre = e1.pre = (T*)pre;
  e0.ldp = e1.ldp = ldp;
  return act == TMAE_ACT_GELU ? launch_gemm<GLDS, T>(nm, W, 0, 0, N, K, xs, e1, M, 1, 1, st)
                              : launch_gemm<GLDS, T>(nm, W, 0, 0, N, K, xs, e0, M, 1, 1, st);
}

template <typename T>
static int linear_t(const void* x, int x_f32, int ldx, int G, int Gs, int off, const void* w, const float* bias,
                    void* y, int y_f32, int ldy, float* y32, int ld32, int M, int N, int K, int act, hipStream_t st,
                    void* pre = nullptr, int ldp = 0) {
  TMAE_REQUIRE(check_k<T>(K) && N % 4 == 0, "tmae_linear_fwd: K=%d must be a multiple of %d and N=%d of 4", K,
               Elt<T>::EPC, N);
  TMAE_REQUIRE(G > 0, "tmae_linear_fwd: row_group must be > 0");
  TMAE_REQUIRE(ldx % Elt<T>::EPC == 0 || x_f32, "tmae_linear_fwd: ldx must keep rows 16-B aligned");
  const T* W = (const T*)w;
  if (x_f32 && sizeof(T) != 4) {
    DenseSrcF32<T> xs{(const float*)x, ldx, M, K, G, Gs, off};
    return linear_epi<T, DenseSrcF32<T>, false>(W, N, K, xs, y, y_f32, ldy, y32, ld32, bias, M, act, st, pre, ldp);
  }
  DenseSrc<T> xs{(const T*)x, ldx, M, K, G, Gs, off, BStride{0, 0}};
  return linear_epi<T, DenseSrc<T>, true>(W, N, K, xs, y, y_f32, ldy, y32, ld32, bias, M, act, st, pre, ldp);
}

#if TMAE_GEMM_TRACE
extern "C" int tmae_gemm_trace_read(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_gemm_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" int tmae_gemm_trace_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_gemm_trace)) != hipSuccess) return 1;
  return hipMemset(p, 0, sizeof(g_gemm_trace)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int tmae_linear_fwd_pre(const void* x, int x_f32, int ldx, int row_group, int group_stride, int row_offset,
                                   const void* w, const float* bias, void* y, int y_f32, int ldy, void* pre, int ldp,
                                   int M, int N, int K, int act, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    return linear_t<bf16>(x, x_f32, ldx, row_group, group_stride, row_offset, w, bias, y, y_f32, ldy, nullptr, 0, M,
                          N, K, act, st, pre, ldp);
  return linear_t<float>(x, 1, ldx, row_group, group_stride, row_offset, w, bias, y, 1, ldy, nullptr, 0, M, N, K, act,
                         st, pre, ldp);
}

template <typename T>
static int resid_out_t(const void* x, int ldx, const void* w, const float* bias, const float* r, float* out, int ld,
                       int M, int N, int K, hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(K) && N % 4 == 0, "tmae_linear_residual_out: bad K=%d / N=%d", K, N);
  DenseSrc<T> xs{(const T*)x, ldx, M, K, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_linear_residual_out", (const T*)w, 0, 0, N, K, xs, EpiResidualOut{r, out, ld, bias},
                              M, 1, 1, st);
}

extern "C" int tmae_linear_residual_out(const void* x, int ldx, const void* w, const float* bias, const float* resid,
                                        float* out, int ld, int M, int N, int K, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return resid_out_t<bf16>(x, ldx, w, bias, resid, out, ld, M, N, K, (hipStream_t)stream);
  return resid_out_t<float>(x, ldx, w, bias, resid, out, ld, M, N, K, (hipStream_t)stream);
}

extern "C" int tmae_linear_fwd(const void* x, int x_f32, int ldx, int row_group, int group_stride, int row_offset,
                               const void* w, const float* bias, void* y, int y_f32, int ldy, float* y32, int ld32,
                               int M, int N, int K, int act, int dtype, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    return linear_t<bf16>(x, x_f32, ldx, row_group, group_stride, row_offset, w, bias, y, y_f32, ldy, y32, ld32, M,
                          N, K, act, st);
  return linear_t<float>(x, 1, ldx, row_group, group_stride, row_offset, w, bias, y, 1, ldy, nullptr, 0, M, N, K,
                         act, st);
}

template <typename T>
static int resid_t(const void* x, int ldx, const void* w, const float* bias, float* r, int ldr, int M, int N, int K,
                   hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(K) && N % 4 == 0, "tmae_linear_residual_fwd: bad K=%d / N=%d", K, N);
  DenseSrc<T> xs{(const T*)x, ldx, M, K, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_linear_residual_fwd", (const T*)w, 0, 0, N, K, xs, EpiResidual{r, ldr, bias}, M,
                              1, 1, st);
}

extern "C" int tmae_linear_residual_fwd(const void* x, int ldx, const void* w, const float* bias, float* resid,
                                        int ldr, int M, int N, int K, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return resid_t<bf16>(x, ldx, w, bias, resid, ldr, M, N, K, (hipStream_t)stream);
  return resid_t<float>(x, ldx, w, bias, resid, ldr, M, N, K, (hipStream_t)stream);
}

// ------------------------------------------------------------------ patch embed (kept patches only)
template <typename T>
static int patch_t(const float* imgs, const int64_t* ids, const void* w, const float* bias, const float* pos,
                   float* tok, int n, int C, int H, int W, int P, int D, int L, int keep, hipStream_t st) {
  const int G = W / P;
  TMAE_REQUIRE(H == W && H % P == 0 && G * G == L, "tmae_patch_embed_fwd: image %dx%d, patch %d, L=%d mismatch", H,
               W, P, L);
  TMAE_REQUIRE(P > 0 && D % 4 == 0, "tmae_patch_embed_fwd: patch %d / dim %d unsupported", P, D);
  // weight rows hold Kw = C*P*P rounded up to a multiple of 8 (zero tail: ViT-H's 588 -> 592)
  const int K = C * P * P, Kw = (K + 7) / 8 * 8;
  PatchSrc<T> xs{imgs, ids, L, keep, C, H, W, P, G, n * keep, K};
  return launch_gemm<false, T>("tmae_patch_embed_fwd", (const T*)w, 0, 0, D, Kw, xs,
                               EpiPatchEmbed{tok, bias, pos, ids, L, keep, D}, n * keep, 1, 1, st);
}

extern "C" int tmae_patch_embed_fwd(const float* imgs, const int64_t* ids_shuffle, const void* w, const float* bias,
                                    const float* pos, float* tokens, int n, int C, int H, int W, int patch, int D,
                                    int L, int keep, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return patch_t<bf16>(imgs, ids_shuffle, w, bias, pos, tokens, n, C, H, W, patch, D, L, keep, (hipStream_t)stream);
  return patch_t<float>(imgs, ids_shuffle, w, bias, pos, tokens, n, C, H, W, patch, D, L, keep, (hipStream_t)stream);
}

// the same GEMM over patches gathered beforehand (tmae_patch_gather: [n*keep][Kw] in T): the LDS-DMA kernel
// instead of the register-staged f32 -> T conversion on load; same MFMA k-order, so the same tokens
template <typename T>
static int patch_gathered_t(const void* patches, const int64_t* ids, const void* w, const float* bias, const float* pos,
                            float* tok, int n, int Kw, int D, int L, int keep, hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(Kw) && D % 4 == 0, "tmae_patch_embed_gathered: K=%d / dim %d unsupported", Kw, D);
  DenseSrc<T> xs{(const T*)patches, Kw, n * keep, Kw, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_patch_embed_gathered", (const T*)w, 0, 0, D, Kw, xs,
                              EpiPatchEmbed{tok, bias, pos, ids, L, keep, D}, n * keep, 1, 1, st);
}

extern "C" int tmae_patch_embed_gathered(const void* patches, const int64_t* ids_shuffle, const void* w,
                                         const float* bias, const float* pos, float* tokens, int n, int Kw, int D,
                                         int L, int keep, int dtype, void* stream) {
  if (dtype == TMAE_BF16)
    return patch_gathered_t<bf16>(patches, ids_shuffle, w, bias, pos, tokens, n, Kw, D, L, keep, (hipStream_t)stream);
  return patch_gathered_t<float>(patches, ids_shuffle, w, bias, pos, tokens, n, Kw, D, L, keep, (hipStream_t)stream);
}

// ------------------------------------------------------------------ decoder embed / pred
template <typename T>
static int dec_embed_t(const void* x, int x_f32, const void* w, const float* bias, const float* pos,
                       const int64_t* ids, float* out, int n, int ntok, int L, int Din, int D, hipStream_t st) {
  TMAE_REQUIRE(check_k<T>(Din) && D % 4 == 0, "tmae_decoder_embed_fwd: bad dims %d -> %d", Din, D);
  TMAE_REQUIRE(ntok >= 1 && ntok <= L + 1, "tmae_decoder_embed_fwd: ntok=%d, L=%d", ntok, L);
  EpiDecoderEmbed epi{out, bias, pos, ids, L, ntok, D};
  if (x_f32 && sizeof(T) != 4) {
    DenseSrcF32<T> xs{(const float*)x, Din, n * ntok, Din, 1 << 30, 0, 0};
    return launch_gemm<false, T>("tmae_decoder_embed_fwd", (const T*)w, 0, 0, D, Din, xs, epi, n * ntok, 1, 1, st);
  }
  DenseSrc<T> xs{(const T*)x, Din, n * ntok, Din, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_decoder_embed_fwd", (const T*)w, 0, 0, D, Din, xs, epi, n * ntok, 1, 1, st);
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
  DenseSrc<T> xs{(const T*)x, Din, n * L, Din, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_decoder_pred_fwd", (const T*)w, 0, 0, N, Din, xs,
                              EpiUnpatchify{imgs, bias, L, G, P, C, H, W}, n * L, 1, 1, st);
}

template <typename T>
static int dec_pred_cp_t(const void* x, const void* w, const float* bias, float* imgs, int n, int L, int Din, int C,
                         int H, int W, int P, hipStream_t st) {
  const int G = W / P;
  const int N = P * P * C;
  TMAE_REQUIRE(H == W && G * G == L && check_k<T>(Din) && P % 8 == 0 && W % 4 == 0,
               "tmae_decoder_pred_cp_fwd: bad geometry (patch must be a multiple of 8)");
  DenseSrc<T> xs{(const T*)x, Din, n * L, Din, 1 << 30, 0, 0, BStride{0, 0}};
  return launch_gemm<true, T>("tmae_decoder_pred_cp_fwd", (const T*)w, 0, 0, N, Din, xs,
                              EpiUnpatchifyCP{imgs, bias, L, G, P, C, H, W}, n * L, 1, 1, st);
}

extern "C" int tmae_decoder_pred_cp_fwd(const void* x, const void* w, const float* bias, float* imgs, int n, int L,
                                        int Din, int C, int H, int W, int patch, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return dec_pred_cp_t<bf16>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
  return dec_pred_cp_t<float>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
}

extern "C" int tmae_decoder_pred_fwd(const void* x, const void* w, const float* bias, float* imgs, int n, int L,
                                     int Din, int C, int H, int W, int patch, int dtype, void* stream) {
  if (dtype == TMAE_BF16) return dec_pred_t<bf16>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
  return dec_pred_t<float>(x, w, bias, imgs, n, L, Din, C, H, W, patch, (hipStream_t)stream);
}

// ------------------------------------------------------------------ diagnostics
extern "C" int tmae_gemm_plan(int M, int N, int K, int batch, int dtype, char* out, int len) {
  TMAE_REQUIRE(out != nullptr && len > 0 && M >= 0 && N >= 0 && K >= 0 && batch >= 1, "tmae_gemm_plan: bad arguments");
  const bool bf = dtype == TMAE_BF16;
  const TileChoice tc = choose_tile(M, N, K, batch, bf);
  snprintf(out, len, "glds<%s,%dx%d,%dw,BK%dx2>", bf ? "bf16" : "f32", tc.bn, tc.bm, tc.nw, bf ? 64 : 32);
  return TMAE_OK;
}
