// Training-step kernels of the MCM hot path (reference MCM.forward + RateDistortionLoss backward, driven by
// utils/engine.py:75-91): weight/data-gradient GEMMs, LayerNorm / GELU / entropy-model backward, layout
// glue of the encoder/decoder, and the optimizer (Adam over flat buffers, clip_grad_norm_).
// Entry points and the reference computation each differentiates: include/tmae.h ("training").
#include "gemm_tn.h"

static int tmae_wgrad_reduce(const float* ws, int splits, int M, int N, float* out, long long base, long long sm,
                             long long sc, long long st, int cp, int accumulate, const float* bws, float* bias_out,
                             int bias_accumulate, hipStream_t s, int nb = 1, long long s_out = 0,
                             long long s_bias = 0);
static int colsum_into(const void* x, int x_dtype, int ld, int rows, int C, int row_group, int group_stride,
                       int row_offset, float* work, long long work_elems, float* out, int accumulate, hipStream_t st);
static int tmae_ln_fold(const float* part, int waves, int D, float* dg, float* db, int accumulate, hipStream_t st);

// ================================================================== helpers
// gelu_grad / gelu_grad2: common.h (shared with the fused slice-stack backward, lic_stack.hip)

// ================================================================== weight gradients (split-K TN GEMM)
template <typename T>
static int wgrad_t(const tmae_wgrad_args& a0, hipStream_t st) {
  const int e = Elt<T>::EPC;
  const int nb = a0.nb > 1 ? a0.nb : 1;
  if (nb > 1 && sizeof(T) == 4) {
    // the f32 parity path: one launch per problem (same per-problem sums as the bf16 batched launch's plan)
    for (int j = 0; j < nb; ++j) {
      tmae_wgrad_args b = a0;
      b.nb = 1;
      b.a = (const T*)a0.a + j * a0.s_a;
      b.b = (const T*)a0.b + j * a0.s_b;
      if (a0.b2) b.b2 = (const T*)a0.b2 + j * a0.s_b2;
      b.out = a0.out + j * a0.s_out;
      if (a0.bias_out) b.bias_out = a0.bias_out + j * a0.s_bias;
      const int rc = wgrad_t<T>(b, st);
      if (rc != TMAE_OK) return rc;
    }
    return TMAE_OK;
  }
  const tmae_wgrad_args& a = a0;
  TMAE_REQUIRE(a.M % e == 0 && a.N % e == 0 && a.lda % e == 0, "tmae_wgrad: M=%d / N=%d / lda must be multiples of %d",
               a.M, a.N, e);
  TMAE_REQUIRE(a.a_G > 0 && a.o_cp > 0, "tmae_wgrad: bad row group / column period");
  const bool bf = sizeof(T) == 2;
  const TnPlan p = tn_plan(a.M, a.N, a.K, bf, a.slot_div, nb);
  const long long slabs = (long long)nb * p.splits * a.M * a.N;
  TMAE_REQUIRE(slabs + (long long)nb * p.splits * a.M <= a.work_elems, "tmae_wgrad: workspace too small (%lld < %lld)",
               a.work_elems, slabs + (long long)nb * p.splits * a.M);
  // bias column sums: in the bf16 kernel (slabs [nb][splits][M] after the partial tiles); the f32 parity path
  // runs the column-sum kernels on A after the GEMM
  float* bws = (a.bias_out && bf) ? a.work + slabs : nullptr;
  // KDenseSrc::addr_in forms element offsets in 32-bit unsigned arithmetic: the last source row the K range
  // reaches, times the stride, plus the columns, must stay below 2^32 elements
  auto last_elem = [&](int G, int Gs, int off, int ld, int cols) -> unsigned long long {
    const long long k = std::max(a.K - 1, 0);
    const long long sk = G < a.K ? (k / G) * (long long)Gs + off + (k % G) : (long long)off + k;
    return (unsigned long long)sk * (unsigned long long)ld + (unsigned long long)cols;
  };
  TMAE_REQUIRE(last_elem(a.a_G, a.a_Gs, a.a_off, a.lda, a.M) < (1ull << 32),
               "tmae_wgrad: operand A spans 2^32 elements or more (32-bit source offsets)");
  KDenseSrc<T> as{(const T*)a.a, a.lda, a.M, a.a_G, a.a_Gs, a.a_off};
  as.sb = a.s_a;
  int rc;
  if (a.b_conv) {
    TMAE_REQUIRE(a.b_Cin % e == 0 && a.b_c1 % e == 0 && a.ldb % e == 0, "tmae_wgrad: conv channels");
    TMAE_REQUIRE(a.N == 9 * a.b_Cin, "tmae_wgrad: N must be 9 * Cin for a 3x3 conv");
    TMAE_REQUIRE(a.b_stride == 1 || a.b_stride == 2, "tmae_wgrad: stride %d", a.b_stride);
    KConvSrc<T> bs;
    bs.x1 = (const T*)a.b; bs.x2 = (const T*)a.b2; bs.c1 = a.b_c1; bs.ld1 = a.ldb; bs.ld2 = a.b_ld2; bs.Cin = a.b_Cin;
    bs.H = a.b_H; bs.W = a.b_W; bs.stride = a.b_stride;
    bs.Ho = (a.b_H + 2 - 3) / a.b_stride + 1; bs.Wo = (a.b_W + 2 - 3) / a.b_stride + 1; bs.cols = a.N;
    bs.sb1 = a.s_b; bs.sb2 = a.s_b2;
    rc = bf ? launch_tn_bf16(p, as, bs, a.work, bws, a.M, a.N, a.K, st, nb)
            : launch_tn_f32(p, as, bs, a.work, a.M, a.N, a.K, st);
  } else {
    TMAE_REQUIRE(a.ldb % e == 0 && a.b_G > 0, "tmae_wgrad: ldb");
    TMAE_REQUIRE(last_elem(a.b_G, a.b_Gs, a.b_off, a.ldb, a.N) < (1ull << 32),
                 "tmae_wgrad: operand B spans 2^32 elements or more (32-bit source offsets)");
    KDenseSrc<T> bs{(const T*)a.b, a.ldb, a.N, a.b_G, a.b_Gs, a.b_off};
    bs.sb = a.s_b;
    rc = bf ? launch_tn_bf16(p, as, bs, a.work, bws, a.M, a.N, a.K, st, nb)
            : launch_tn_f32(p, as, bs, a.work, a.M, a.N, a.K, st);
  }
  if (rc != TMAE_OK) return rc;
  rc = tmae_wgrad_reduce(a.work, p.splits, a.M, a.N, a.out, a.o_base, a.o_sm, a.o_sc, a.o_st, a.o_cp, a.accumulate,
                         bws, bws ? a.bias_out : nullptr, a.bias_accumulate, st, nb, a.s_out, a.s_bias);
  if (rc != TMAE_OK || !a.bias_out || bf) return rc;
  // f32: the partial-tile slabs are consumed; their space is the column sums' workspace
  return colsum_into(a.a, TMAE_F32, a.lda, a.K, a.M, a.a_G, a.a_Gs, a.a_off, a.work, a.work_elems, a.bias_out,
                     a.bias_accumulate, st);
}

// fixed-order sum over the split slabs, scattered into the parameter's layout:
// dst = base + m*sm + (n % cp)*sc + (n / cp)*st   (dense [M][N]: sm=N, sc=1, cp=N; conv [co][ci][3][3]
// from columns tap*Cin + ci: sm=cin_total*9, sc=9, st=1, cp=Cin, base=ci_off*9; transposed: sm=1, sc=M)
// Threads past M*N fold the bias slab [splits][M] (same fixed order) into bias_out.
// Each thread sums 4 consecutive elements (16-B loads of every split slab; N is a multiple of 8, so the 4 share
// a row); threads past M*N/4 fold the bias slab [splits][M] (same fixed order) into bias_out.
__global__ void __launch_bounds__(256)
tn_reduce_kernel(const float* __restrict__ ws, int splits, int M, int N, float* __restrict__ out, long long base,
                 long long sm, long long sc, long long st, int cp, int accumulate, const float* __restrict__ bws,
                 float* __restrict__ bias_out, int bias_accumulate, long long s_out, long long s_bias) {
  const long long t = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long tot = (long long)M * N, tot4 = tot >> 2;
  // problem blockIdx.y of a batched weight gradient: its slabs, its bias slab, its parameter
  ws += (size_t)blockIdx.y * splits * tot;
  out += blockIdx.y * s_out;
  if (bws) bws += (size_t)blockIdx.y * splits * M;
  if (bias_out) bias_out += blockIdx.y * s_bias;
  if (t >= tot4) {
    const long long m = t - tot4;
    if (!bias_out || m >= M) return;
    // split order as one add at a time; the loads of 16 (then 4) splits in flight together (a dependent load per
    // split made these last threads the kernel's tail: ~0.3 us of latency per split)
    float s = 0.0f;
    int k = 0;
    for (; k + 16 <= splits; k += 16) {
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = bws[(size_t)(k + j) * M + m];
#pragma unroll
      for (int j = 0; j < 16; ++j) s += v[j];
    }
    for (; k + 4 <= splits; k += 4) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = bws[(size_t)(k + j) * M + m];
#pragma unroll
      for (int j = 0; j < 4; ++j) s += v[j];
    }
    for (; k < splits; ++k) s += bws[(size_t)k * M + m];
    bias_out[m] = bias_accumulate ? bias_out[m] + s : s;
    return;
  }
  const long long i = 4 * t;
  const int m = (int)(i / N), n = (int)(i - (long long)m * N);
  // the slabs are summed in split order (bitwise the same as one load and add at a time), but the loads of
  // 16 (then 4) splits are issued together: with a few dozen splits over a small output (the LIC convs: 36 splits,
  // ~25 blocks) one dependent load per split left the kernel latency-bound
  f32x4 s = load4f(ws + i);
  int k = 1;
  for (; k + 16 <= splits; k += 16) {
    f32x4 v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = load4f(ws + (size_t)(k + j) * tot + i);
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
  }
  for (; k + 4 <= splits; k += 4) {
    f32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = load4f(ws + (size_t)(k + j) * tot + i);
#pragma unroll
    for (int j = 0; j < 4; ++j) s += v[j];
  }
  for (; k < splits; ++k) s += load4f(ws + (size_t)k * tot + i);
  if (sc == 1 && (n % cp) + 4 <= cp) {  // 4 consecutive destinations (dense layouts, and a conv's channel run)
    float* d = out + base + m * sm + (long long)(n % cp) + (long long)(n / cp) * st;
    if (accumulate) {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] += s[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = s[e];
    }
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ne = n + e;
    const long long d = base + m * sm + (long long)(ne % cp) * sc + (long long)(ne / cp) * st;
    out[d] = accumulate ? out[d] + s[e] : s[e];
  }
}

static int tmae_wgrad_reduce(const float* ws, int splits, int M, int N, float* out, long long base, long long sm,
                             long long sc, long long st, int cp, int accumulate, const float* bws, float* bias_out,
                             int bias_accumulate, hipStream_t s, int nb, long long s_out, long long s_bias) {
  const long long tot = (long long)M * N / 4 + (bias_out ? M : 0);  // threads (N % 8 == 0: wgrad_t)
  if (tot == 0) return TMAE_OK;
  hipLaunchKernelGGL(tn_reduce_kernel, dim3((unsigned)((tot + 255) / 256), nb), dim3(256), 0, s, ws, splits, M, N, out,
                     base, sm, sc, st, cp, accumulate, bws, bias_out, bias_accumulate, s_out, s_bias);
  TMAE_LAUNCH_CHECK("tmae_wgrad");
}

extern "C" int tmae_wgrad(const tmae_wgrad_args* a, int dtype, void* stream) {
  TMAE_REQUIRE(a != nullptr && a->a && a->b && a->work && a->out, "tmae_wgrad: null argument");
  if (a->M == 0 || a->N == 0) return TMAE_OK;
  if (dtype == TMAE_BF16) return wgrad_t<bf16>(*a, (hipStream_t)stream);
  return wgrad_t<float>(*a, (hipStream_t)stream);
}

extern "C" long long tmae_wgrad_workspace(int M, int N, int K, int dtype) {
  const TnPlan p = tn_plan(M, N, K, dtype == TMAE_BF16);
  return (long long)p.splits * M * N + (long long)p.splits * M;  // partial tiles + bias column-sum slab
}

/* the same for nb problems of one batched launch at 1 / slot_div of the slots */
extern "C" long long tmae_wgrad_workspace_nb(int M, int N, int K, int dtype, int slot_div, int nb) {
  nb = nb > 1 ? nb : 1;
  const TnPlan p = tn_plan(M, N, K, dtype == TMAE_BF16, slot_div, nb);
  const TnPlan p1 = tn_plan(M, N, K, dtype == TMAE_BF16);
  const long long one = (long long)p1.splits * M * N + (long long)p1.splits * M;  // the f32 per-problem path
  return std::max((long long)nb * p.splits * ((long long)M * N + M), one);
}

// ================================================================== data gradients (NT core on transposed weights)
// out = acc * (pre ? gelu'(pre) : 1) in OT; acc32 (optional) += the same value in f32
template <typename OT, typename PT> struct EpiDgrad {
  OT* out;
  int ldo;
  const PT* pre;
  int ldp;
  float* acc;
  int lda;
  long long s_out = 0, s_pre = 0;  // element offsets of problem b1's out / pre (batched launches)
  __device__ void batch(int b1, int) {
    out += b1 * s_out;
    if (pre) pre += b1 * s_pre;
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    if (pre) {
      const f32x4 p = load4f(pre + (size_t)m * ldp + n);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] *= gelu_grad(p[j]);
    }
    if (out) store4(out + (size_t)m * ldo + n, v);
    if (acc) {
      float* q = acc + (size_t)m * lda + n;
      store4(q, load4f(q) + v);
    }
  }
  // epilogue_lds hook: the GELU inputs and the f32 accumulator rows one block ahead of the stores
  struct Pre { f32x4 p0, p1, a0, a1; };
  __device__ Pre fetch(int m, int n) const {
    Pre q;
    if (pre) load8f(pre + (size_t)m * ldp + n, q.p0, q.p1);
    if (acc) load8f(acc + (size_t)m * lda + n, q.a0, q.a1);
    return q;
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi, const Pre& q) const {
    if (pre) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const f32x2 gl = gelu_grad2((f32x2){q.p0[j], q.p0[j + 1]}), gh = gelu_grad2((f32x2){q.p1[j], q.p1[j + 1]});
        lo[j] *= gl.x; lo[j + 1] *= gl.y; hi[j] *= gh.x; hi[j + 1] *= gh.y;
      }
    }
    if (out) store8(out + (size_t)m * ldo + n, lo, hi);
    if (acc) store8(acc + (size_t)m * lda + n, q.a0 + lo, q.a1 + hi);
  }};

// columns [0, lim0) -> d0, [lim0, lim1) -> d1, [lim1, lim2) -> d2; each f32 +=  (conv input = channel concat)
struct EpiRoute3 {
  float* d[3];
  int ld[3];
  int lim[3];
  __device__ void batch(int, int) {}
  __device__ __forceinline__ float* at(int m, int n) const {
    if (n < lim[0]) return d[0] + (size_t)m * ld[0] + n;
    if (n < lim[1]) return d[1] + (size_t)m * ld[1] + (n - lim[0]);
    return d[2] + (size_t)m * ld[2] + (n - lim[1]);
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    float* q = at(m, n);
    store4(q, load4f(q) + v);
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const {
    operator()(m, n, lo);
    operator()(m, n + 4, hi);
  }
};

template <typename T>
static int dgrad_linear_t(const void* dy, int ldy, int G, int Gs, int off, const void* wt, int M, int N, int K, void* out,
                          int out_f32, int ldo, const void* pre, int ldp, float* acc, int lda, hipStream_t st) {
  TMAE_REQUIRE(N % Elt<T>::EPC == 0 && K % 4 == 0 && ldy % Elt<T>::EPC == 0 && G > 0,
               "tmae_dgrad_linear: N=%d / K=%d / ldy unsupported", N, K);
  DenseSrc<T> xs{(const T*)dy, ldy, M, N, G, Gs, off, BStride{0, 0}};
  const char* nm = "tmae_dgrad_linear";
  if (out_f32 || !out) {
    EpiDgrad<float, T> e{(float*)out, ldo, (const T*)pre, ldp, acc, lda};
    return launch_gemm<true, T>(nm, (const T*)wt, 0, 0, K, N, xs, e, M, 1, 1, st);
  }
  EpiDgrad<T, T> e{(T*)out, ldo, (const T*)pre, ldp, acc, lda};
  return launch_gemm<true, T>(nm, (const T*)wt, 0, 0, K, N, xs, e, M, 1, 1, st);
}

extern "C" int tmae_dgrad_linear(const void* dy, int ldy, int row_group, int group_stride, int row_offset,
                                 const void* wt, int M, int N, int K, void* out, int out_f32, int ldo, const void* pre,
                                 int ldp, float* acc32, int ld32, int dtype, void* stream) {
  TMAE_REQUIRE(dy && wt && (out || acc32), "tmae_dgrad_linear: null argument");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16)
    return dgrad_linear_t<bf16>(dy, ldy, row_group, group_stride, row_offset, wt, M, N, K, out, out_f32, ldo, pre, ldp,
                                acc32, ld32, st);
  return dgrad_linear_t<float>(dy, ldy, row_group, group_stride, row_offset, wt, M, N, K, out, 1, ldo, pre, ldp, acc32,
                               ld32, st);
}

// ---------------------------------------------------------------- conv dgrad: transposed-conv row source
// row m = input pixel (b, iy, ix); k = tap * Cout + co reads dY at the output pixel that saw (iy, ix)
// through tap (ky, kx): oy = (iy + 1 - ky) / stride when integral and in range, else zero.
template <typename T> struct ConvTSrc {
  const T* dy;
  int ldy, Cout, H, W, Ho, Wo, stride, rows, K;
  float inv_cout;
  long long s_dy;  // element offset of problem b1's dy (batched launches)
  struct Row { int b; int iy; int ix; bool ok; };
  __device__ void batch(int b1, int) { dy += b1 * s_dy; }
  __device__ Row row(int m) const {
    if (m >= rows) return {0, 0, 0, false};
    const int hw = H * W;
    const int b = m / hw, rem = m - b * hw;
    const int iy = rem / W;
    return {b, iy, rem - iy * W, true};
  }
  __device__ const void* addr_k(const Row& r, int k) const {
    if (!r.ok || k >= K) return g_tmae_zero_page;
    int tap = (int)((float)k * inv_cout);
    if (tap * Cout > k) --tap;
    if ((tap + 1) * Cout <= k) ++tap;
    const int co = k - tap * Cout;
    const int ky = (tap * 11) >> 5;
    int ty = r.iy + 1 - ky, tx = r.ix + 1 - (tap - 3 * ky);
    if (ty < 0 || tx < 0) return g_tmae_zero_page;
    if (stride == 2) {
      if ((ty | tx) & 1) return g_tmae_zero_page;
      ty >>= 1;
      tx >>= 1;
    }
    if (ty >= Ho || tx >= Wo) return g_tmae_zero_page;
    return dy + ((size_t)(r.b * Ho + ty) * Wo + tx) * ldy + co;
  }
  __device__ const void* addr(const Row& r, int kt, int c) const {
    return addr_k(r, kt * 8 * Elt<T>::EPC + c * Elt<T>::EPC);
  }
  __device__ uint4 load(const Row& r, int kt, int c) const { return *reinterpret_cast<const uint4*>(addr(r, kt, c)); }
  // K iterator for the LDS-DMA ring (as ConvSrc::It, gemm_core.h): a lane's chunk carries its tap and output
  // channel from K-step to K-step; the tap's dy pointer is rebuilt only when the chunk crosses into the next tap.
  // Same addresses as addr_k.
  struct It { const T* p; int co, tap, b, iy, ix; bool ok, in; };
  __device__ void it_tap(It& it) const {
    const int ky = (it.tap * 11) >> 5;  // tap / 3 for tap < 9
    int ty = it.iy + 1 - ky, tx = it.ix + 1 - (it.tap - 3 * ky);
    bool in = it.ok && it.tap < 9 && ty >= 0 && tx >= 0;
    if (stride == 2) {
      in = in && !((ty | tx) & 1);
      ty >>= 1;
      tx >>= 1;
    }
    in = in && ty < Ho && tx < Wo;
    it.in = in;
    it.p = dy + ((size_t)(it.b * Ho + (in ? ty : 0)) * Wo + (in ? tx : 0)) * ldy;
  }
  __device__ It iter(const Row& r, int c) const {
    It it{nullptr, c * Elt<T>::EPC, 0, r.b, r.iy, r.ix, r.ok && Cout > 0, false};
    while (it.ok && it.co >= Cout) { it.co -= Cout; ++it.tap; }
    it_tap(it);
    return it;
  }
  __device__ const void* next(It& it) const {
    const void* a = it.in ? (const void*)(it.p + it.co) : (const void*)g_tmae_zero_page;
    it.co += 8 * Elt<T>::EPC;
    if (it.co >= Cout && it.ok) {
      do { it.co -= Cout; ++it.tap; } while (it.co >= Cout);
      it_tap(it);
    }
    return a;
  }
};

template <typename T>
static int conv_dgrad_t(const tmae_conv_dgrad_args& a, hipStream_t st) {
  const int e = Elt<T>::EPC;
  TMAE_REQUIRE(a.cout % e == 0 && a.ldy % e == 0 && a.cin % 4 == 0, "tmae_conv_dgrad: channels %d -> %d", a.cout,
               a.cin);
  TMAE_REQUIRE(a.stride == 1 || a.stride == 2, "tmae_conv_dgrad: stride %d", a.stride);
  ConvTSrc<T> xs;
  xs.dy = (const T*)a.dy; xs.ldy = a.ldy; xs.Cout = a.cout; xs.H = a.H; xs.W = a.W; xs.stride = a.stride;
  xs.Ho = (a.H + 2 - 3) / a.stride + 1; xs.Wo = (a.W + 2 - 3) / a.stride + 1;
  xs.rows = a.n * a.H * a.W; xs.K = 9 * a.cout; xs.inv_cout = 1.0f / (float)a.cout;
  xs.s_dy = a.s_dy;
  const int M = xs.rows, K = xs.K, N = a.cin;
  const int nb = a.nb > 1 ? a.nb : 1;
  const char* nm = "tmae_conv_dgrad";
  TMAE_REQUIRE(nb <= 65535 && (nb == 1 || !a.acc[0]), "tmae_conv_dgrad: batched (nb = %d) launches take no routes",
               nb);
  if (a.acc[0]) {
    TMAE_REQUIRE(a.lim[0] % 8 == 0 && a.lim[1] % 8 == 0 && a.lim[2] == a.cin && a.lim[0] <= a.lim[1] &&
                     a.lim[1] <= a.lim[2],
                 "tmae_conv_dgrad: route limits");
    TMAE_REQUIRE((a.lim[1] == a.lim[0] || a.acc[1]) && (a.lim[2] == a.lim[1] || a.acc[2]),
                 "tmae_conv_dgrad: route destination missing");
    EpiRoute3 r;
    for (int i = 0; i < 3; ++i) { r.d[i] = a.acc[i]; r.ld[i] = a.ld_acc[i]; r.lim[i] = a.lim[i]; }
    return launch_gemm<true, T>(nm, (const T*)a.wd, 0, 0, N, K, xs, r, M, 1, 1, st);
  }
  if (a.out_f32) {
    EpiDgrad<float, T> g{(float*)a.out, a.ldo, (const T*)a.pre, a.ldp, nullptr, 0, a.s_out, a.s_pre};
    return launch_gemm<true, T>(nm, (const T*)a.wd, a.s_wd, 0, N, K, xs, g, M, nb, 1, st);
  }
  EpiDgrad<T, T> g{(T*)a.out, a.ldo, (const T*)a.pre, a.ldp, nullptr, 0, a.s_out, a.s_pre};
  return launch_gemm<true, T>(nm, (const T*)a.wd, a.s_wd, 0, N, K, xs, g, M, nb, 1, st);
}

extern "C" int tmae_conv_dgrad(const tmae_conv_dgrad_args* a, int dtype, void* stream) {
  TMAE_REQUIRE(a && a->dy && a->wd && (a->out || a->acc[0]), "tmae_conv_dgrad: null argument");
  if (dtype == TMAE_BF16) return conv_dgrad_t<bf16>(*a, (hipStream_t)stream);
  TMAE_REQUIRE(a->out_f32 || a->acc[0], "tmae_conv_dgrad: the f32 path writes f32 outputs");
  return conv_dgrad_t<float>(*a, (hipStream_t)stream);
}

// ================================================================== weight re-layout + cast
// dst (contiguous, dims d0..d3) = cast(src[i0*s0 + i1*s1 + i2*s2 + i3*s3]); src f32
template <typename OT>
__global__ void __launch_bounds__(256)
relayout_kernel(const float* __restrict__ src, OT* __restrict__ dst, int d1, int d2, int d3, long long s0, long long s1,
                long long s2, long long s3, long long total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  long long r = i;
  const int i3 = (int)(r % d3); r /= d3;
  const int i2 = (int)(r % d2); r /= d2;
  const int i1 = (int)(r % d1);
  const long long i0 = r / d1;
  dst[i] = to_out<OT>(src[i0 * s0 + i1 * s1 + i2 * s2 + i3 * s3]);
}

// 2-D transpose-cast through LDS: dst[c][r] = src[r][c] (src rows of ld_src floats), R rows, C columns
template <typename OT>
__global__ void __launch_bounds__(256)
transpose_kernel(const float* __restrict__ src, int ld_src, OT* __restrict__ dst, int R, int C) {
  __shared__ float t[32][33];
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int k = ty; k < 32; k += 8) {
    const int r = r0 + k, c = c0 + tx;
    t[k][tx] = (r < R && c < C) ? src[(size_t)r * ld_src + c] : 0.0f;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int c = c0 + k, r = r0 + tx;
    if (c < C && r < R) dst[(size_t)c * R + r] = to_out<OT>(t[tx][k]);
  }
}

extern "C" int tmae_relayout(const float* src, void* dst, int dst_dtype, int d0, int d1, int d2, int d3, long long s0,
                             long long s1, long long s2, long long s3, void* stream) {
  TMAE_REQUIRE(src && dst && d0 >= 0 && d1 > 0 && d2 > 0 && d3 > 0, "tmae_relayout: bad arguments");
  const long long total = (long long)d0 * d1 * d2 * d3;
  if (total == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  // a plain 2-D transpose (dst[i0][i3] = src[i3 * ld + i0]) goes through the LDS tile: coalesced both ways
  if (d1 == 1 && d2 == 1 && s0 == 1 && s3 >= d0) {
    const dim3 grid(ceil_div(d0, 32), ceil_div(d3, 32));
    if (dst_dtype == TMAE_BF16)
      hipLaunchKernelGGL(transpose_kernel<bf16>, grid, dim3(256), 0, st, src, (int)s3, (bf16*)dst, d3, d0);
    else
      hipLaunchKernelGGL(transpose_kernel<float>, grid, dim3(256), 0, st, src, (int)s3, (float*)dst, d3, d0);
    TMAE_LAUNCH_CHECK("tmae_relayout");
  }
  const dim3 grid((unsigned)((total + 255) / 256));
  if (dst_dtype == TMAE_BF16)
    hipLaunchKernelGGL(relayout_kernel<bf16>, grid, dim3(256), 0, st, src, (bf16*)dst, d1, d2, d3, s0, s1, s2, s3, total);
  else
    hipLaunchKernelGGL(relayout_kernel<float>, grid, dim3(256), 0, st, src, (float*)dst, d1, d2, d3, s0, s1, s2, s3,
                       total);
  TMAE_LAUNCH_CHECK("tmae_relayout");
}

// multi-tensor form: table[t] = {src, dst, dst_dtype | mode << 8, d1, d2, d3, s0, s1, s2, s3, total, first_chunk}
// (int64), followed by the row t of every chunk (a block reads its row index instead of searching first_chunk).
// One launch re-lays out every weight whose version moved (the optimizer step), instead of one launch per weight
// and layout.  Modes (host-chosen):
//   0  32768-element chunks: plain casts as 16-B vectors (4 rounds of 4 x 8 elements per thread), anything else
//      as a strided gather;
//   1  2-D transpose dst[c][r] = src[r * s3 + c] (R = d3 source rows, C = total / R; s1 != 0: also the plain cast
//      into s1 = a second destination [R][C], one read for both layouts): 64 x 64 LDS tiles, coalesced
//      both ways (nn.Linear data-gradient operands W^T; the conv data-gradient layout [Cin][3][3][Cout], which is
//      the transpose of the weight seen as [Cout][Cin * 9]); 16-B loads and 4-row (8-B bf16) stores when the
//      source rows are 16-B aligned and R % 4 == 0 (scalar 4-B loads / 2-B stores ran at ~2 TB/s);
//   2  per-row [A][B] -> [B][A] (conv weight [Cout][Cin][3][3] -> [Cout][3][3][Cin]: A = Cin = d3, B = 9): one row
//      per chunk through LDS (A * B <= 8192); 16-B loads and 8-B bf16 stores when A % 4 == 0 and aligned;
//   3  tmae_lic_stack's fragment order of a channel range of a conv weight (below; 256 units of 9 x 8 elements per
//      chunk);
//   4  the same for the transposed, tap-flipped weight (the fused stack backward's).
template <typename OT>
__device__ __forceinline__ void relayout_store(void* dst, size_t i, float v) { reinterpret_cast<OT*>(dst)[i] = to_out<OT>(v); }

__global__ void __launch_bounds__(256)
relayout_multi_kernel(const long long* __restrict__ tab, int nt) {
  __shared__ __attribute__((aligned(16))) float sm[8192];
  const long long b = blockIdx.x;
  // the table's per-chunk row index (after the nt rows): one load instead of a search of the rows
  const int lo = (int)tab[12 * (long long)nt + b];
  const long long* e = tab + 12 * lo;
  const float* src = (const float*)e[0];
  void* dstp = (void*)e[1];
  const unsigned d1 = (unsigned)e[3], d2 = (unsigned)e[4], d3 = (unsigned)e[5];
  const long long s0 = e[6], s1 = e[7], s2 = e[8], s3 = e[9];
  const unsigned total = (unsigned)e[10];  // < 2^31 (host check)
  const int mode = (int)(e[2] >> 8);
  const bool to_bf16 = (e[2] & 255) == TMAE_BF16;
  const unsigned chunk = (unsigned)(b - e[11]);
  const int tid = threadIdx.x;
  if (mode == 1) {
    const unsigned R = d3, C = total / d3;
    const unsigned ntc = (C + 63) / 64;
    const unsigned r0 = (chunk / ntc) * 64, c0 = (chunk % ntc) * 64;
    const int tx = tid & 63, ty = tid >> 6;
    // s1 != 0: also the plain cast of the same source into dst2 [R][C] (a weight needed both ways reads once)
    void* dst2 = (void*)s1;
    const bool vec = to_bf16 && (R & 3u) == 0 && (C & 3u) == 0 && (s3 & 3) == 0 && (((unsigned long long)src) & 15) == 0 &&
                     (((unsigned long long)dstp) & 7) == 0 && (((unsigned long long)dst2) & 7) == 0;
    if (vec) {
      // loads: a thread reads 4 consecutive columns of rows ty4, ty4 + 16, .. (16 rows of 16 float4 per pass)
      const int c4 = 4 * (tid & 15), ty4 = tid >> 4;
#pragma unroll
      for (int k = ty4; k < 64; k += 16) {
        const unsigned r = r0 + k, c = c0 + c4;
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        if (r < R && c < C) {
          v = load4f(src + (size_t)r * s3 + c);  // C % 4 == 0: all 4 columns valid
          if (dst2) {
            bf16x4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) o[j] = (bf16)v[j];
            *reinterpret_cast<bf16x4*>((bf16*)dst2 + (size_t)r * C + c) = o;
          }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) sm[k * 65 + c4 + j] = v[j];
      }
      __syncthreads();
      // stores: a thread writes 4 consecutive destination columns (source rows r4..r4+3) of dst row c
      const int r4 = 4 * (tid & 15), kc = tid >> 4;
#pragma unroll
      for (int k = kc; k < 64; k += 16) {
        const unsigned c = c0 + k, r = r0 + r4;
        if (c < C && r < R) {  // R % 4 == 0: all 4 rows valid
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = (bf16)sm[(r4 + j) * 65 + k];
          *reinterpret_cast<bf16x4*>((bf16*)dstp + (size_t)c * R + r) = o;
        }
      }
      return;
    }
#pragma unroll 4
    for (int k = ty; k < 64; k += 4) {
      const unsigned r = r0 + k, c = c0 + tx;
      const float v = (r < R && c < C) ? src[(size_t)r * s3 + c] : 0.0f;
      sm[k * 65 + tx] = v;
      if (dst2 && r < R && c < C) {
        if (to_bf16) relayout_store<bf16>(dst2, (size_t)r * C + c, v);
        else relayout_store<float>(dst2, (size_t)r * C + c, v);
      }
    }
    __syncthreads();
#pragma unroll 4
    for (int k = ty; k < 64; k += 4) {
      const unsigned c = c0 + k, r = r0 + tx;
      if (c < C && r < R) {
        if (to_bf16) relayout_store<bf16>(dstp, (size_t)c * R + r, sm[tx * 65 + k]);
        else relayout_store<float>(dstp, (size_t)c * R + r, sm[tx * 65 + k]);
      }
    }
    return;
  }
  if (mode == 2) {
    const unsigned A = d3, B = d1 * d2, n = A * B, r = chunk;
    if (to_bf16 && (A & 3u) == 0 && (s0 & 3) == 0 && (((unsigned long long)src) & 15) == 0 &&
        (((unsigned long long)dstp) & 7) == 0) {
      // 16-B loads into LDS; each store is 4 consecutive destination elements (a..a+3 of tap t, 8 B)
      for (unsigned i = tid; i < n / 4; i += 256) *reinterpret_cast<f32x4*>(sm + 4 * i) = load4f(src + (size_t)r * s0 + 4 * i);
      __syncthreads();
      const unsigned A4 = A / 4;
      bf16* ob = (bf16*)dstp + (size_t)r * n;
      for (unsigned idx = tid; idx < B * A4; idx += 256) {
        const unsigned t = idx / A4, a = 4 * (idx - t * A4);
        bf16x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (bf16)sm[(a + j) * B + t];
        *reinterpret_cast<bf16x4*>(ob + (size_t)t * A + a) = o;
      }
      return;
    }
    for (unsigned i = tid; i < n; i += 256) sm[i] = src[(size_t)r * s0 + i];
    __syncthreads();
    const size_t ob = (size_t)r * n;
    for (unsigned t = 0; t < B; ++t)
      for (unsigned a = tid; a < A; a += 256) {
        if (to_bf16) relayout_store<bf16>(dstp, ob + (size_t)t * A + a, sm[a * B + t]);
        else relayout_store<float>(dstp, ob + (size_t)t * A + a, sm[a * B + t]);
      }
    return;
  }
  if (mode == 3 || mode == 4) {
    // tmae_lic_stack's MFMA fragment order [tap][k-step][fragment][lane = 16 fq + fr][8] of a 3x3 conv weight.
    //   3: weight [Cout = d1][Cin_tot = d2][3][3] (f32), input channels [d3, d3 + s0): element e of lane (fq, fr),
    //      fragment f, k-step kc, tap t = W[16 f + fr][d3 + 32 kc + 8 fq + e][t] (ops.pack_lic_stack_weight);
    //   4: the transposed, tap-flipped weight (the data gradient's: input = the forward's Cout = d1 channels, output =
    //      its Cin = d2): W[32 kc + 8 fq + e][16 f + fr][8 - t] (ops.pack_lic_stack_weight_t).
    // Zero past the channel ranges.  One thread = one (k-step, fragment, lane) unit, all 9 taps: its source values
    // are 9 consecutive floats per element (the taps), read once; it writes one 16-B run per tap, a wave 1 KiB per
    // tap.  (An element per thread read each source line once per tap through 4-B gathers: 1.1 TB/s.)
    const unsigned nfr = mode == 3 ? (d1 + 15) / 16 : (d2 + 15) / 16;
    const unsigned nkc = mode == 3 ? ((unsigned)s0 + 31) / 32 : (d1 + 31) / 32;
    const unsigned units = nkc * nfr * 64u;
    const unsigned u = chunk * 256u + (unsigned)tid;
    if (u >= units) return;
    const unsigned lane = u & 63u, fk = u >> 6, f = fk % nfr, kc = fk / nfr;
    const unsigned fr = lane & 15u, fq = lane >> 4;
    float v[9][8];
    if (mode == 3) {
      const unsigned cout = d1, cin_tot = d2, c_lo = d3, cn = (unsigned)s0;
      const unsigned co = 16 * f + fr, ci0 = 32 * kc + 8 * fq;
      const float* rowp = src + ((size_t)co * cin_tot + c_lo + ci0) * 9;
      if (co < cout && ci0 + 8 <= cn && ((((unsigned long long)rowp) & 15) == 0)) {
        f32x4 q[18];
#pragma unroll
        for (int k = 0; k < 18; ++k) q[k] = load4f(rowp + 4 * k);
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int t = 0; t < 9; ++t) v[t][j] = q[(9 * j + t) >> 2][(9 * j + t) & 3];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int t = 0; t < 9; ++t) v[t][j] = (co < cout && ci0 + j < cn) ? rowp[9 * j + t] : 0.0f;
      }
    } else {
      const unsigned cout = d1, cin = d2;
      const unsigned ci = 16 * f + fr, co0 = 32 * kc + 8 * fq;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = ci < cin && co0 + j < cout;
        const float* tp = src + ((size_t)(co0 + j) * cin + ci) * 9;
#pragma unroll
        for (int t = 0; t < 9; ++t) v[t][j] = ok ? tp[8 - t] : 0.0f;
      }
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const size_t o = ((size_t)(t * nkc + kc) * nfr + f) * 512 + (size_t)lane * 8;
      const f32x4 lo4 = f32x4{v[t][0], v[t][1], v[t][2], v[t][3]}, hi4 = f32x4{v[t][4], v[t][5], v[t][6], v[t][7]};
      if (to_bf16) store8((bf16*)e[1] + o, lo4, hi4);
      else store8((float*)e[1] + o, lo4, hi4);
    }
    return;
  }
  const unsigned base = chunk * 32768u;
  // a plain cast (contiguous source, 16-B aligned ends): 16 x 8 elements per thread (4 rounds of 4 x 8 in
  // flight), vector loads and stores
  const bool dense = (d3 == 1 || s3 == 1) && (d2 == 1 || s2 == (long long)d3) && (d1 == 1 || s1 == (long long)d2 * d3) &&
                     s0 == (long long)d1 * d2 * d3 &&
                     ((((unsigned long long)src) | ((unsigned long long)e[1])) & 15) == 0;
  if (dense && (total & 7u) == 0) {
    for (unsigned rb = base; rb < base + 32768u && rb < total; rb += 8192u) {
      f32x4 lo4[4], hi4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned i = rb + 2048u * u + 8u * tid;
        if (i < total) load8f(src + i, lo4[u], hi4[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned i = rb + 2048u * u + 8u * tid;
        if (i >= total) break;
        if (to_bf16) store8((bf16*)e[1] + i, lo4[u], hi4[u]);
        else store8((float*)e[1] + i, lo4[u], hi4[u]);
      }
    }
    return;
  }
  // general strided gather: 32-bit index arithmetic (64-bit division is a long VALU sequence)
  for (unsigned k = tid; k < 32768u; k += 256u) {
    const unsigned i = base + k;
    if (i >= total) break;
    unsigned r = i;
    const unsigned i3 = r % d3; r /= d3;
    const unsigned i2 = r % d2; r /= d2;
    const unsigned i1 = r % d1;
    const unsigned i0 = r / d1;
    const float v = src[(long long)i0 * s0 + (long long)i1 * s1 + (long long)i2 * s2 + (long long)i3 * s3];
    if (to_bf16) ((bf16*)e[1])[i] = (bf16)v;
    else ((float*)e[1])[i] = v;
  }
}

extern "C" int tmae_relayout_multi(const long long* table, int ntensors, long long nchunks, void* stream) {
  TMAE_REQUIRE(table && ntensors > 0, "tmae_relayout_multi: bad arguments");
  if (nchunks <= 0) return TMAE_OK;
  hipLaunchKernelGGL(relayout_multi_kernel, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, table, ntensors);
  TMAE_LAUNCH_CHECK("tmae_relayout_multi");
}

// ================================================================== column sums (bias gradients)
// part[split][c] = sum over this split's rows r of x[src_row(r)][c]; src_row = (r / G) * Gs + off + r % G
template <typename T>
__global__ void __launch_bounds__(256)
colsum_partial_kernel(const T* __restrict__ x, int ld, int rows, int C, int G, int Gs, int off, int rows_per_split,
                      float* __restrict__ part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_split, r1 = min(rows, r0 + rows_per_split);
  float s = 0.0f;
  for (int r = r0; r < r1; ++r) {
    const int sr = (r / G) * Gs + off + (r % G);
    s += (float)x[(size_t)sr * ld + c];
  }
  part[(size_t)blockIdx.y * C + c] = s;
}

// vector form: a thread owns 8 consecutive columns (one 16-B bf16 load per row, two for f32) and walks its
// rows with an incremental row-group map (no division per row); needs C, ld multiples of 8
template <typename T>
__global__ void __launch_bounds__(256)
colsum_partial8_kernel(const T* __restrict__ x, int ld, int rows, int C, int G, int Gs, int off, int rows_per_split,
                       float* __restrict__ part) {
  const int c = (blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= C) return;
  const int r0 = blockIdx.y * rows_per_split, r1 = min(rows, r0 + rows_per_split);
  f32x4 s0{0.f, 0.f, 0.f, 0.f}, s1{0.f, 0.f, 0.f, 0.f};
  int q = r0 / G, rem = r0 - (r0 / G) * G;
  for (int r = r0; r < r1; ++r) {
    f32x4 lo, hi;
    load8f(x + (size_t)(q * Gs + off + rem) * ld + c, lo, hi);
    s0 += lo;
    s1 += hi;
    if (++rem == G) { rem = 0; ++q; }
  }
  store8(part + (size_t)blockIdx.y * C + c, s0, s1);
}

// fold [rows][C] partials over rows: 64 columns x 16 row-lanes per block, fixed-order LDS tree
// (deterministic); columns [0, split) -> out0[c], [split, split2) -> out1[c - split], [split2, C) ->
// out2[c - split2]
__global__ void __launch_bounds__(1024)
fold_rows_kernel(const float* __restrict__ part, int rows, int C, float* __restrict__ out0, float* __restrict__ out1,
                 int split, int accumulate, float* __restrict__ out2, int split2) {
  // 16 columns x 64 row-lanes per block (64-B row segments): four times the blocks and a quarter of the
  // serial rows per thread of a 64 x 16 block -- these folds are latency-bound (C = 2304 gave 36 blocks)
  __shared__ float red[64][17];
  const int cx = threadIdx.x & 15, ry = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cx;
  float s = 0.0f;
  if (c < C)
    for (int r = ry; r < rows; r += 64) s += part[(size_t)r * C + c];
  red[ry][cx] = s;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) {
    if (ry < o) red[ry][cx] += red[ry + o][cx];
    __syncthreads();
  }
  if (ry == 0 && c < C) {
    float* dst = c < split ? out0 + c : c < split2 ? out1 + (c - split) : out2 + (c - split2);
    *dst = accumulate ? *dst + red[0][cx] : red[0][cx];
  }
}

static void fold_rows(const float* part, int rows, int C, float* out0, float* out1, int split, int accumulate,
                      hipStream_t st, float* out2 = nullptr, int split2 = -1) {
  hipLaunchKernelGGL(fold_rows_kernel, dim3(ceil_div(C, 16)), dim3(1024), 0, st, part, rows, C, out0, out1, split,
                     accumulate, out2, split2 < 0 ? C : split2);
}

extern "C" int tmae_colsum(const void* x, int x_dtype, int ld, int rows, int C, int row_group, int group_stride,
                           int row_offset, float* work, long long work_elems, float* out, int accumulate, void* stream) {
  return colsum_into(x, x_dtype, ld, rows, C, row_group, group_stride, row_offset, work, work_elems, out, accumulate,
                     (hipStream_t)stream);
}

static int colsum_into(const void* x, int x_dtype, int ld, int rows, int C, int row_group, int group_stride,
                       int row_offset, float* work, long long work_elems, float* out, int accumulate, hipStream_t st) {
  TMAE_REQUIRE(x && out && work && row_group > 0, "tmae_colsum: bad arguments");
  if (C == 0) return TMAE_OK;
  int splits = std::max(1, std::min(256, rows / 32));
  while ((long long)splits * C > work_elems && splits > 1) splits /= 2;
  TMAE_REQUIRE((long long)splits * C <= work_elems, "tmae_colsum: workspace too small");
  const int rps = ceil_div(std::max(rows, 1), splits);
  if (C % 8 == 0 && ld % 8 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)work & 15) == 0) {
    const dim3 grid8(ceil_div(C / 8, 256), splits);
    if (x_dtype == TMAE_BF16)
      hipLaunchKernelGGL(colsum_partial8_kernel<bf16>, grid8, dim3(256), 0, st, (const bf16*)x, ld, rows, C, row_group,
                         group_stride, row_offset, rps, work);
    else
      hipLaunchKernelGGL(colsum_partial8_kernel<float>, grid8, dim3(256), 0, st, (const float*)x, ld, rows, C,
                         row_group, group_stride, row_offset, rps, work);
    fold_rows(work, splits, C, out, out, C, accumulate, st);
    TMAE_LAUNCH_CHECK("tmae_colsum");
  }
  const dim3 grid(ceil_div(C, 256), splits);
  if (x_dtype == TMAE_BF16)
    hipLaunchKernelGGL(colsum_partial_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)x, ld, rows, C, row_group,
                       group_stride, row_offset, rps, work);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<float>, grid, dim3(256), 0, st, (const float*)x, ld, rows, C, row_group,
                       group_stride, row_offset, rps, work);
  fold_rows(work, splits, C, out, out, C, accumulate, st);
  TMAE_LAUNCH_CHECK("tmae_colsum");
}

// ================================================================== LayerNorm backward
// x rows remapped like the forward (source row sr = (r / G) * Gs + off + r % G); dy dense [rows][D] f32.
// dx lands at row sr of dx32 (f32; + dres[sr] when given) and of dxop (operand dtype copy, optional).
// Waves walk rows r = wave, wave + nwaves, ... with the NEXT row's x / dy / dres loads issued before this row's
// reductions (one row's latency hidden under the previous row's math; 8 waves per CU); dgamma / dbeta (and RS)
// partials stay in registers per wave, are summed over the workgroup's 4 waves in LDS and written once per
// workgroup -> part [workgroup][np * D] (np = 2, or 3 with RS: also the column sums of dres, the bias gradient
// of the Linear whose output the residual adds: fc2 before norm2's input gradient, proj before norm1's).
template <typename OT, int VPL, bool RS>
__global__ void __launch_bounds__(256)
layernorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ dy,
                     const float* __restrict__ dres, float* __restrict__ dx32, OT* __restrict__ dxop, int rows, int D,
                     int G, int Gs, int off, float eps, float* __restrict__ part) {
  constexpr int NP = RS ? 3 : 2;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][NP * D]
  const int lane = threadIdx.x & 63, wl = threadIdx.x >> 6;
  const int nwaves = gridDim.x * 4;
  const int nch = D >> 2;
  f32x4 dg[VPL], db[VPL], gm[VPL], dr[VPL];
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    dg[i] = db[i] = dr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int c = lane + 64 * i;
    gm[i] = c < nch ? load4f(gamma + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 v[VPL], g[VPL], rv[VPL];
  auto load_row = [&](int r, f32x4 (&vv)[VPL], f32x4 (&gg)[VPL], f32x4 (&rr)[VPL]) {
    const int sr = (r / G) * Gs + off + (r % G);
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      const bool ok = c < nch && r < rows;
      vv[i] = ok ? load4f(x + (size_t)sr * D + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
      gg[i] = ok ? load4f(dy + (size_t)r * D + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
      rr[i] = (ok && dres) ? load4f(dres + (size_t)sr * D + 4 * c) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  int r = blockIdx.x * 4 + wl;
  if (r < rows) load_row(r, v, g, rv);
  for (; r < rows; r += nwaves) {
    const int sr = (r / G) * Gs + off + (r % G);
    f32x4 vn[VPL], gn[VPL], rn[VPL];
    if (r + nwaves < rows) load_row(r + nwaves, vn, gn, rn);  // next row in flight under this one
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
    s = wave_allsum(s);
    const float mean = s / (float)D;
    float q = 0.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float d = v[i][j] - mean;
          q += d * d;
        }
      }
    }
    q = wave_allsum(q);
    const float rstd = 1.0f / sqrtf(q / (float)D + eps);
    float sa = 0.0f, sb = 0.0f;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xh = (v[i][j] - mean) * rstd;
          v[i][j] = xh;
          const float gg = g[i][j] * gm[i][j];
          sa += gg;
          sb += gg * xh;
          dg[i][j] += g[i][j] * xh;
          db[i][j] += g[i][j];
        }
      }
    }
    sa = wave_allsum(sa);
    sb = wave_allsum(sb);
    sa /= (float)D;
    sb /= (float)D;
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        f32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = rstd * (g[i][j] * gm[i][j] - sa - v[i][j] * sb);
        if (dres) {
          o += rv[i];
          if (RS) dr[i] += rv[i];
        }
        store4(dx32 + (size_t)sr * D + 4 * c, o);
        if (dxop) store4(dxop + (size_t)sr * D + 4 * c, o);
      }
    }
#pragma unroll
    for (int i = 0; i < VPL; ++i) {
      v[i] = vn[i];
      g[i] = gn[i];
      rv[i] = rn[i];
    }
  }
  // the workgroup's four wave partials -> one row of part (fixed order: deterministic)
  float* rw = red + (size_t)wl * NP * D;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      *reinterpret_cast<f32x4*>(rw + 4 * c) = dg[i];
      *reinterpret_cast<f32x4*>(rw + D + 4 * c) = db[i];
      if (RS) *reinterpret_cast<f32x4*>(rw + 2 * D + 4 * c) = dr[i];
    }
  }
  __syncthreads();
  float* pw = part + (size_t)blockIdx.x * NP * D;
  for (int e = threadIdx.x; e < NP * D; e += 256)
    pw[e] = ((red[e] + red[NP * D + e]) + red[2 * NP * D + e]) + red[3 * NP * D + e];
}

static int tmae_ln_fold(const float* part, int waves, int D, float* dg, float* db, float* drs, int accumulate,
                        hipStream_t st) {
  if (drs) fold_rows(part, waves, 3 * D, dg, db, D, accumulate, st, drs, 2 * D);
  else fold_rows(part, waves, 2 * D, dg, db, D, accumulate, st);
  TMAE_LAUNCH_CHECK("tmae_layernorm_bwd");
}

extern "C" int tmae_layernorm_bwd(const float* x, const float* gamma, const float* dy, const float* dres, float* dx32,
                                  void* dxop, int op_dtype, int rows, int D, int row_group, int group_stride,
                                  int row_offset, float eps, float* work, long long work_elems, float* dgamma,
                                  float* dbeta, float* dres_colsum, int accumulate, void* stream) {
  TMAE_REQUIRE(D % 4 == 0 && D <= 2048 && row_group > 0, "tmae_layernorm_bwd: D=%d", D);
  TMAE_REQUIRE(x && gamma && dy && dx32 && work && dgamma && dbeta, "tmae_layernorm_bwd: null argument");
  TMAE_REQUIRE(!dres_colsum || dres, "tmae_layernorm_bwd: dres_colsum needs dres");
  hipStream_t st = (hipStream_t)stream;
  const int np = dres_colsum ? 3 : 2;  // partial blocks per workgroup
  // 2 workgroups (8 waves) per CU, each wave ~rows / 2048 rows; fewer when the rows are few
  int wgs = std::max(1, std::min(512, ceil_div(std::max(rows, 1), 4 * 2)));
  while ((long long)wgs * np * D > work_elems && wgs > 1) wgs /= 2;
  TMAE_REQUIRE((long long)wgs * np * D <= work_elems, "tmae_layernorm_bwd: workspace too small");
  const int waves = wgs;  // partial rows for the fold
  const int vpl = ceil_div(D / 4, 64);
  const dim3 grid(wgs);
  const size_t lds = (size_t)4 * np * D * sizeof(float);
  TMAE_REQUIRE(lds <= 160 * 1024, "tmae_layernorm_bwd: D=%d needs %zu B of LDS (160 KiB per workgroup)", D, lds);
#define TMAE_LNB(OT, V)                                                                                               \
  if (dres_colsum)                                                                                                    \
    hipLaunchKernelGGL((layernorm_bwd_kernel<OT, V, true>), grid, dim3(256), lds, st, x, gamma, dy, dres, dx32,         \
                       (OT*)dxop, rows, D, row_group, group_stride, row_offset, eps, work);                           \
  else                                                                                                                \
    hipLaunchKernelGGL((layernorm_bwd_kernel<OT, V, false>), grid, dim3(256), lds, st, x, gamma, dy, dres, dx32,        \
                       (OT*)dxop, rows, D, row_group, group_stride, row_offset, eps, work)
#define TMAE_LNB_V(OT)          \
  if (vpl <= 1) TMAE_LNB(OT, 1);  \
  else if (vpl <= 2) TMAE_LNB(OT, 2); \
  else if (vpl <= 3) TMAE_LNB(OT, 3); \
  else if (vpl <= 4) TMAE_LNB(OT, 4); \
  else TMAE_LNB(OT, 8)
  if (op_dtype == TMAE_BF16) {
    TMAE_LNB_V(bf16);
  } else {
    TMAE_LNB_V(float);
  }
#undef TMAE_LNB_V
#undef TMAE_LNB
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    tmae_set_error(TMAE_EHIP, "tmae_layernorm_bwd: launch failed: %s", hipGetErrorString(e));
    return TMAE_EHIP;
  }
  return tmae_ln_fold(work, waves, D, dgamma, dbeta, dres_colsum, accumulate, st);
}

// ================================================================== elementwise backward pieces
// subpel_conv3x3 backward (compressai PixelShuffle(2) after the conv, then GELU): dpre [n*H*W][4c] (conv
// channel co = c*4 + i*2 + j of pixel (y, x)) = dy_ps[(2y+i, 2x+j)][c] * gelu'(pre_ps) (pre optional)
template <typename GT, typename T>
__global__ void __launch_bounds__(256)
unshuffle_bwd_kernel(const GT* __restrict__ dy, int ldy, const T* __restrict__ pre, int ldp, T* __restrict__ out,
                     int n, int H, int W, int C4) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long total = (long long)n * H * W * C4;
  if (i >= total) return;
  const int co = (int)(i % C4);
  const long long m = i / C4;
  const int hw = H * W;
  const int b = (int)(m / hw), rem = (int)(m - (long long)b * hw);
  const int y = rem / W, x = rem - y * W;
  const int c = co >> 2, si = (co >> 1) & 1, sj = co & 1;
  const size_t at = ((size_t)(b * 2 * H + 2 * y + si) * 2 * W + 2 * x + sj);
  float g = (float)dy[at * ldy + c];
  if (pre) g *= gelu_grad((float)pre[at * ldp + c]);
  out[i] = to_out<T>(g);
}

extern "C" int tmae_unshuffle_bwd(const void* dy, int dy_f32, int ldy, const void* pre, int ldp, void* out, int n,
                                  int H, int W, int C4, int dtype, void* stream) {
  TMAE_REQUIRE(C4 % 4 == 0, "tmae_unshuffle_bwd: channels %d", C4);
  const long long total = (long long)n * H * W * C4;
  if (total == 0) return TMAE_OK;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
#define TMAE_UB(GT, T)                                                                                             \
  hipLaunchKernelGGL((unshuffle_bwd_kernel<GT, T>), grid, dim3(256), 0, st, (const GT*)dy, ldy, (const T*)pre, ldp, \
                     (T*)out, n, H, W, C4)
  if (dtype == TMAE_BF16) {
    if (dy_f32) TMAE_UB(float, bf16);
    else TMAE_UB(bf16, bf16);
  } else {
    TMAE_UB(float, float);
  }
#undef TMAE_UB
  TMAE_LAUNCH_CHECK("tmae_unshuffle_bwd");
}

// y = gelu(pre) elementwise backward: out = dy * gelu'(pre)  (layers whose dgrad epilogue cannot fuse it)
template <typename GT, typename T>
__global__ void __launch_bounds__(256)
gelu_bwd_kernel(const GT* __restrict__ dy, const T* __restrict__ pre, T* __restrict__ out, long long total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  out[i] = to_out<T>((float)dy[i] * gelu_grad((float)pre[i]));
}

extern "C" int tmae_gelu_bwd(const void* dy, int dy_f32, const void* pre, void* out, long long total, int dtype,
                             void* stream) {
  if (total <= 0) return TMAE_OK;
  const dim3 grid((unsigned)((total + 255) / 256));
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16) {
    if (dy_f32)
      hipLaunchKernelGGL((gelu_bwd_kernel<float, bf16>), grid, dim3(256), 0, st, (const float*)dy, (const bf16*)pre,
                         (bf16*)out, total);
    else
      hipLaunchKernelGGL((gelu_bwd_kernel<bf16, bf16>), grid, dim3(256), 0, st, (const bf16*)dy, (const bf16*)pre,
                         (bf16*)out, total);
  } else {
    hipLaunchKernelGGL((gelu_bwd_kernel<float, float>), grid, dim3(256), 0, st, (const float*)dy, (const float*)pre,
                       (float*)out, total);
  }
  TMAE_LAUNCH_CHECK("tmae_gelu_bwd");
}

// last lrp_transform conv (MCM.py:779-783): y_hat = y_hat_pre + 0.5 tanh(t).  g = g32 (f32, optional) + g16
// (operand dtype, optional) is the y_hat gradient; dt = g * 0.5 (1 - tanh(t)^2) (operand dtype) and
// gsum = g (f32, optional: the y_hat_pre gradient the GaussianConditional backward continues with)
template <typename T>
__global__ void __launch_bounds__(256)
lrp_bwd_kernel(const float* __restrict__ g32, int ld32, const float* __restrict__ g32b, int ld32b,
               const T* __restrict__ g16, int ld16, const float* __restrict__ t, int ldt, T* __restrict__ dt, int lddt,
               float* __restrict__ gsum, int ldgs, int rows, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * C) return;
  const int m = i / C, c = i - m * C;
  float g = g32 ? g32[(size_t)m * ld32 + c] : 0.0f;
  if (g32b) g += g32b[(size_t)m * ld32b + c];
  if (g16) g += (float)g16[(size_t)m * ld16 + c];
  const float th = tanhf(t[(size_t)m * ldt + c]);
  dt[(size_t)m * lddt + c] = to_out<T>(g * 0.5f * (1.0f - th * th));
  if (gsum) gsum[(size_t)m * ldgs + c] = g;
}

extern "C" int tmae_lrp_bwd(const float* g32, int ld32, const float* g32b, int ld32b, const void* g16, int ld16,
                            const float* t, int ldt, void* dt, int lddt, float* gsum, int ldgs, int rows, int C,
                            int dtype, void* stream) {
  if (rows * C == 0) return TMAE_OK;
  const dim3 grid(ceil_div(rows * C, 256));
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(lrp_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, g32, ld32, g32b, ld32b,
                       (const bf16*)g16, ld16, t, ldt, (bf16*)dt, lddt, gsum, ldgs, rows, C);
  else
    hipLaunchKernelGGL(lrp_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, g32, ld32, g32b, ld32b,
                       (const float*)g16, ld16, t, ldt, (float*)dt, lddt, gsum, ldgs, rows, C);
  TMAE_LAUNCH_CHECK("tmae_lrp_bwd");
}

// strided 2-D copy of rows x cols elements (esz = 2 or 4 bytes)
template <typename E>
__global__ void __launch_bounds__(256)
copy2d_kernel(const E* __restrict__ src, int lds, E* __restrict__ dst, int ldd, int rows, int cols) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)rows * cols) return;
  const int r = (int)(i / cols), c = (int)(i - (long long)r * cols);
  dst[(size_t)r * ldd + c] = src[(size_t)r * lds + c];
}

extern "C" int tmae_copy2d(const void* src, int lds, void* dst, int ldd, int rows, int cols, int esz, void* stream) {
  TMAE_REQUIRE(esz == 2 || esz == 4, "tmae_copy2d: element size %d", esz);
  const long long total = (long long)rows * cols;
  if (total <= 0) return TMAE_OK;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (esz == 2)
    hipLaunchKernelGGL(copy2d_kernel<uint16_t>, grid, dim3(256), 0, (hipStream_t)stream, (const uint16_t*)src, lds,
                       (uint16_t*)dst, ldd, rows, cols);
  else
    hipLaunchKernelGGL(copy2d_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, (const float*)src, lds,
                       (float*)dst, ldd, rows, cols);
  TMAE_LAUNCH_CHECK("tmae_copy2d");
}

// GaussianConditional backward for one slice (compressai 1.2.4 _likelihood + LowerBound semantics,
// MCM.py:771-776).  Element (pixel m, channel c) of slice channel ch = yoff + c.
//   lik = LB_1e-9( Phi((1/2 - v)/s) - Phi((-1/2 - v)/s) ),  v = |x~ - mu|,  s = LB_0.11(sigma)
//   x~ = y + noise (train) | round(y - mu) + mu (eval);  y_hat_pre = STE(y - mu) + mu
// LowerBound backward passes the gradient where x >= bound or grad < 0.
// Outputs: dy (f32, +=), dmu / dsigma (operand dtype, [m][ldd]).
template <typename T>
__global__ void __launch_bounds__(256)
gc_bwd_kernel(const float* __restrict__ y, int ldy, int yoff, const float* __restrict__ mu,
              const float* __restrict__ sigma, int ld_ms, const float* __restrict__ noise, int Mtot,
              const float* __restrict__ glik, const float* __restrict__ gyp, int ldg, float* __restrict__ dy, int lddy,
              T* __restrict__ dmu, T* __restrict__ dsig, int ldd, int n, int HW, int sw) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * HW * sw) return;
  const int m = i / sw, c = i - m * sw;
  const int ch = yoff + c;
  const int b = m / HW, pix = m - b * HW;
  const size_t nchw = ((size_t)b * Mtot + ch) * HW + pix;
  const float yv = y[(size_t)m * ldy + ch];
  const float mv = mu[(size_t)m * ld_ms + c];
  const float sr = sigma[(size_t)m * ld_ms + c];
  const float xt = noise ? yv + noise[nchw] : rintf(yv - mv) + mv;
  const float s = fmaxf(sr, 0.11f);
  const float dd = xt - mv;
  const float v = fabsf(dd);
  const float a = (0.5f - v) / s, bb = (-0.5f - v) / s;
  const float k = -0.70710678118654752440f;
  const float lik = 0.5f * erfcf(k * a) - 0.5f * erfcf(k * bb);
  float g = glik ? glik[nchw] : 0.0f;
  if (!(lik >= 1e-9f || g < 0.0f)) g = 0.0f;
  const float inv_sqrt2pi = 0.39894228040143267794f;
  const float pa = inv_sqrt2pi * expf(-0.5f * a * a), pb = inv_sqrt2pi * expf(-0.5f * bb * bb);
  const float dv = g * (pb - pa) / s;
  float ds = g * (bb * pb - a * pa) / s;
  if (!(sr >= 0.11f || ds < 0.0f)) ds = 0.0f;
  const float sg = dd > 0.0f ? 1.0f : (dd < 0.0f ? -1.0f : 0.0f);
  const float ddd = dv * sg;  // d lik / d (x~ - mu)
  float dyv = gyp ? gyp[(size_t)m * ldg + ch] : 0.0f;  // STE path of y_hat_pre
  float dmv = -ddd;
  if (noise) dyv += ddd;
  else dmv += ddd;  // eval: x~ = round(y - mu) + mu moves with mu, round has no gradient
  dy[(size_t)m * lddy + ch] += dyv;
  dmu[(size_t)m * ldd + c] = to_out<T>(dmv);
  dsig[(size_t)m * ldd + c] = to_out<T>(ds);
}

extern "C" int tmae_gc_bwd(const float* y, int ldy, int yoff, const float* mu, const float* sigma, int ld_ms,
                           const float* noise, int Mtot, const float* glik, const float* gyp, int ldg, float* dy,
                           int lddy, void* dmu, void* dsigma, int ldd, int n, int HW, int sw, int dtype, void* stream) {
  const int total = n * HW * sw;
  if (total == 0) return TMAE_OK;
  const dim3 grid(ceil_div(total, 256));
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(gc_bwd_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, y, ldy, yoff, mu, sigma, ld_ms,
                       noise, Mtot, glik, gyp, ldg, dy, lddy, (bf16*)dmu, (bf16*)dsigma, ldd, n, HW, sw);
  else
    hipLaunchKernelGGL(gc_bwd_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, y, ldy, yoff, mu, sigma, ld_ms,
                       noise, Mtot, glik, gyp, ldg, dy, lddy, (float*)dmu, (float*)dsigma, ldd, n, HW, sw);
  TMAE_LAUNCH_CHECK("tmae_gc_bwd");
}

// ================================================================== EntropyBottleneck backward
// compressai 1.2.4 _logits_cumulative / _likelihood (MCM.py:741), per channel c (one workgroup):
//   h = softplus(M0) v + b0; h += tanh(F0) tanh(h); [h = softplus(Ml) h + bl; h += tanh(Fl) tanh(h)] x3;
//   f = softplus(M4) h + b4;  lik = LB_1e-9 |sigmoid(s f(x+1/2)) - sigmoid(s f(x-1/2))|, s = -sign(sum) detached
// Gradients: dz (x = z + noise in training; the STE z_hat adds its own pass-through gz) and every density
// parameter of the channel (softplus' = sigmoid below the threshold 20, tanh' = 1 - tanh^2).
struct EbCh {
  float sp0[3], b0[3], tf0[3];
  float sp[3][9], bl[3][3], tf[3][3];
  float sp4[3], b4;
};
typedef EbCh EbGrad;  // gradient w.r.t. the same packed (transformed) quantities

__device__ __forceinline__ float eb_softplus(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ float eb_softplus_grad(float x) { return x > 20.0f ? 1.0f : 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float eb_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ void eb_load(const tmae_eb_params& p, int c, EbCh& w) {
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    w.sp0[j] = eb_softplus(p.matrix[0][c * 3 + j]);
    w.b0[j] = p.bias[0][c * 3 + j];
    w.tf0[j] = tanhf(p.factor[0][c * 3 + j]);
  }
#pragma unroll
  for (int l = 0; l < 3; ++l) {
#pragma unroll
    for (int e = 0; e < 9; ++e) w.sp[l][e] = eb_softplus(p.matrix[l + 1][c * 9 + e]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      w.bl[l][j] = p.bias[l + 1][c * 3 + j];
      w.tf[l][j] = tanhf(p.factor[l + 1][c * 3 + j]);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) w.sp4[k] = eb_softplus(p.matrix[4][c * 3 + k]);
  w.b4 = p.bias[4][c];
}

// f(v); for upstream gradient go also accumulates the packed-parameter gradients (GR) and df/dv (dv != null).
// gr: the packed gradient sums, EbCh field order (sp0 0, b0 3, tf0 6, sp 9, bl 36, tf 45, sp4 54, b4 57), in a
// plain float array, loops unrolled, GR a template flag rather than a null test: comparing the private array's
// address with null kept the 58 sums in scratch (236 B per lane, every accumulation a scratch read-modify-write)
template <bool GR>
__device__ __forceinline__ float eb_fwd_bwd(const EbCh& w, float v, float go, float* gr, float* dv) {
  float u[4][3], th[4][3], h[4][3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    u[0][j] = w.sp0[j] * v + w.b0[j];
    th[0][j] = tanhf(u[0][j]);
    h[0][j] = u[0][j] + w.tf0[j] * th[0][j];
  }
#pragma unroll
  for (int l = 0; l < 3; ++l) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u[l + 1][i] = (w.sp[l][3 * i] * h[l][0] + w.sp[l][3 * i + 1] * h[l][1] + w.sp[l][3 * i + 2] * h[l][2]) + w.bl[l][i];
      th[l + 1][i] = tanhf(u[l + 1][i]);
      h[l + 1][i] = u[l + 1][i] + w.tf[l][i] * th[l + 1][i];
    }
  }
  const float f = (w.sp4[0] * h[3][0] + w.sp4[1] * h[3][1] + w.sp4[2] * h[3][2]) + w.b4;
  if (!GR && !dv) return f;
  float dh[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    dh[k] = go * w.sp4[k];
    if constexpr (GR) gr[54 + k] += go * h[3][k];
  }
  if constexpr (GR) gr[57] += go;
#pragma unroll
  for (int l = 2; l >= 0; --l) {
    float du[3], dprev[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      du[i] = dh[i] * (1.0f + w.tf[l][i] * (1.0f - th[l + 1][i] * th[l + 1][i]));
      if constexpr (GR) {
        gr[45 + 3 * l + i] += dh[i] * th[l + 1][i];
        gr[36 + 3 * l + i] += du[i];
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        if constexpr (GR) gr[9 + 9 * l + 3 * i + j] += du[i] * h[l][j];
        dprev[j] += w.sp[l][3 * i + j] * du[i];
      }
    }
#pragma unroll
    for (int j = 0; j < 3; ++j) dh[j] = dprev[j];
  }
  float d = 0.0f;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const float du = dh[j] * (1.0f + w.tf0[j] * (1.0f - th[0][j] * th[0][j]));
    if constexpr (GR) {
      gr[6 + j] += dh[j] * th[0][j];
      gr[3 + j] += du;
      gr[j] += du * v;
    }
    d += w.sp0[j] * du;
  }
  if (dv) *dv = d;
  return f;
}

#define EB_NG 58

__global__ void __launch_bounds__(256)
eb_bwd_kernel(tmae_eb_params p, const float* __restrict__ z, const float* __restrict__ noise,
              const float* __restrict__ glik, const float* __restrict__ gzhat, float* __restrict__ dz, int C, int HW,
              int n, tmae_eb_params g, int accumulate) {
  const int c = blockIdx.x;
  EbCh w;
  eb_load(p, c, w);
  const float med = p.quantiles[c * 3 + 1];
  float gf[EB_NG];
#pragma unroll
  for (int k = 0; k < EB_NG; ++k) gf[k] = 0.0f;
  const int total = n * HW;
  for (int e = threadIdx.x; e < total; e += 256) {
    const int b = e / HW, pix = e - b * HW;
    const size_t nhwc = ((size_t)b * HW + pix) * C + c;
    const size_t nchw = ((size_t)b * C + c) * HW + pix;
    const float zv = z[nhwc];
    const float x = noise ? zv + noise[nchw] : rintf(zv - med) + med;
    const float lower = eb_fwd_bwd<false>(w, x - 0.5f, 0.0f, nullptr, nullptr);
    const float upper = eb_fwd_bwd<false>(w, x + 0.5f, 0.0f, nullptr, nullptr);
    const float sum = lower + upper;
    const float s = sum > 0.0f ? -1.0f : (sum < 0.0f ? 1.0f : 0.0f);
    const float su = eb_sigmoid(s * upper), sl = eb_sigmoid(s * lower);
    const float raw = fabsf(su - sl);
    float gl = glik ? glik[nchw] : 0.0f;
    if (!(raw >= 1e-9f || gl < 0.0f)) gl = 0.0f;
    const float sg = su > sl ? 1.0f : (su < sl ? -1.0f : 0.0f);
    const float gu = gl * sg * s * su * (1.0f - su);
    const float glo = -gl * sg * s * sl * (1.0f - sl);
    float dvu = 0.0f, dvl = 0.0f;
    if (gu != 0.0f) eb_fwd_bwd<true>(w, x + 0.5f, gu, gf, &dvu);
    if (glo != 0.0f) eb_fwd_bwd<true>(w, x - 0.5f, glo, gf, &dvl);
    float d = gzhat ? gzhat[nhwc] : 0.0f;  // quantize_ste pass-through (MCM.py:742-744)
    if (noise) d += dvu + dvl;             // eval: x = round(z - med) + med, no gradient to z
    dz[nhwc] = d;
  }
  // workgroup reduction of the 58 parameter gradients
  __shared__ float red[EB_NG][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < EB_NG; ++k) {
    const float v = wave_allsum(gf[k]);
    if (lane == 0) red[k][wv] = v;
  }
  __syncthreads();
  if (threadIdx.x < EB_NG) {
    const int k = threadIdx.x;
    const float v = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    // packed index -> (tensor element, chain rule of softplus / tanh back to the raw parameter)
    float* dst;
    float dval;
    if (k < 3) {
      dst = (float*)g.matrix[0] + c * 3 + k;
      dval = v * eb_softplus_grad(p.matrix[0][c * 3 + k]);
    } else if (k < 6) {
      dst = (float*)g.bias[0] + c * 3 + (k - 3);
      dval = v;
    } else if (k < 9) {
      const float t = tanhf(p.factor[0][c * 3 + k - 6]);
      dst = (float*)g.factor[0] + c * 3 + (k - 6);
      dval = v * (1.0f - t * t);
    } else if (k < 36) {
      const int l = (k - 9) / 9, e = (k - 9) % 9;
      dst = (float*)g.matrix[l + 1] + c * 9 + e;
      dval = v * eb_softplus_grad(p.matrix[l + 1][c * 9 + e]);
    } else if (k < 45) {
      const int l = (k - 36) / 3, j = (k - 36) % 3;
      dst = (float*)g.bias[l + 1] + c * 3 + j;
      dval = v;
    } else if (k < 54) {
      const int l = (k - 45) / 3, j = (k - 45) % 3;
      const float t = tanhf(p.factor[l + 1][c * 3 + j]);
      dst = (float*)g.factor[l + 1] + c * 3 + j;
      dval = v * (1.0f - t * t);
    } else if (k < 57) {
      dst = (float*)g.matrix[4] + c * 3 + (k - 54);
      dval = v * eb_softplus_grad(p.matrix[4][c * 3 + k - 54]);
    } else {
      dst = (float*)g.bias[4] + c;
      dval = v;
    }
    *dst = accumulate ? *dst + dval : dval;
  }
}

extern "C" int tmae_eb_bwd(const tmae_eb_params* params, const float* z, const float* noise, const float* glik,
                           const float* gzhat, float* dz, int n, int C, int HW, const tmae_eb_params* grads,
                           int accumulate, void* stream) {
  TMAE_REQUIRE(params && grads && z && dz, "tmae_eb_bwd: null argument");
  static_assert(sizeof(EbGrad) == EB_NG * sizeof(float), "EbGrad packing");
  if (C == 0) return TMAE_OK;
  hipLaunchKernelGGL(eb_bwd_kernel, dim3(C), dim3(256), 0, (hipStream_t)stream, *params, z, noise, glik, gzhat, dz, C,
                     HW, n, *grads, accumulate);
  TMAE_LAUNCH_CHECK("tmae_eb_bwd");
}

// aux_loss backward (compressai EntropyBottleneck.loss, stop_gradient=True on the density parameters):
// d/dq[c][j] = g * sign(f_c(q[c][j]) - target[j]) * f_c'(q[c][j])
__global__ void __launch_bounds__(256)
eb_aux_bwd_kernel(tmae_eb_params p, const float* __restrict__ target, const float* __restrict__ gout,
                  float* __restrict__ dq, int C, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= C * 3) return;
  const int c = i / 3, j = i - 3 * c;
  EbCh w;
  eb_load(p, c, w);
  float d = 0.0f;
  const float f = eb_fwd_bwd<false>(w, p.quantiles[i], 1.0f, nullptr, &d);
  const float r = f - target[j];
  const float sg = r > 0.0f ? 1.0f : (r < 0.0f ? -1.0f : 0.0f);
  const float v = (gout ? gout[0] : 1.0f) * sg * d;
  dq[i] = accumulate ? dq[i] + v : v;
}

extern "C" int tmae_eb_aux_bwd(const tmae_eb_params* params, const float* target, const float* gout, float* dquantiles,
                               int C, int accumulate, void* stream) {
  TMAE_REQUIRE(params && target && dquantiles, "tmae_eb_aux_bwd: null argument");
  if (C == 0) return TMAE_OK;
  hipLaunchKernelGGL(eb_aux_bwd_kernel, dim3(ceil_div(3 * C, 256)), dim3(256), 0, (hipStream_t)stream, *params, target,
                     gout, dquantiles, C, accumulate);
  TMAE_LAUNCH_CHECK("tmae_eb_aux_bwd");
}

// ================================================================== rate term backward
// bpp = (sum log y + sum log z) / (-ln2 * num_pixels) (rd_loss.py:19-20): dlik = g / (lik * -ln2 * num_pixels)
__global__ void __launch_bounds__(256)
bpp_bwd_kernel(const float* __restrict__ lik, const float* __restrict__ g, float* __restrict__ out, long long n,
               float scale) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  out[i] = g[0] * scale / lik[i];
}

extern "C" int tmae_bpp_bwd(const float* lik, const float* gout, float* dlik, long long n, double num_pixels,
                            void* stream) {
  if (n <= 0) return TMAE_OK;
  hipLaunchKernelGGL(bpp_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, lik, gout,
                     dlik, n, (float)(1.0 / (-0.69314718055994530942 * num_pixels)));
  TMAE_LAUNCH_CHECK("tmae_bpp_bwd");
}

// ================================================================== encoder / decoder glue
// kept-patch im2col (timm PatchEmbed conv16/s16 over the kept patches, MCM.py:615 + gather 585-586):
// out[b*keep + k][(c*P + py)*P + px] = img[b][c][hy*P + py][hx*P + px], patch ids_shuffle[b][k]; rows are Kw =
// C*P*P rounded up to a multiple of 8 values, the tail zero (ViT-H's patch 14: 588 -> 592, the GEMMs' 16-B rows)
template <typename T>
__global__ void __launch_bounds__(256)
patch_gather_kernel(const float* __restrict__ img, const int64_t* __restrict__ ids, T* __restrict__ out, int n, int C,
                    int H, int W, int P, int L, int keep) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int KP = C * P * P, Kw = (KP + 7) / 8 * 8;
  if (i >= (long long)n * keep * Kw) return;
  const int col = (int)(i % Kw);
  if (col >= KP) {
    out[i] = to_out<T>(0.0f);
    return;
  }
  const int row = (int)(i / Kw);
  const int b = row / keep, k = row - b * keep;
  const int p = (int)ids[(size_t)b * L + k];
  const int G = W / P;
  const int hy = p / G, hx = p - hy * G;
  const int c = col / (P * P), rem = col - c * P * P;
  const int py = rem / P, px = rem - py * P;
  out[i] = to_out<T>(img[(((size_t)b * C + c) * H + hy * P + py) * W + hx * P + px]);
}

// the same with 8 consecutive pixels of one patch row per thread (P % 8 == 0): two 16-B loads, one 16-B (bf16) or
// two (f32) stores; one thread per (row, channel, patch row, 8-pixel group)
template <typename T>
__global__ void __launch_bounds__(256)
patch_gather8_kernel(const float* __restrict__ img, const int64_t* __restrict__ ids, T* __restrict__ out, int n, int C,
                     int H, int W, int P, int L, int keep) {
  const int per_row = C * P * (P / 8);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n * keep * per_row) return;
  const int row = i / per_row, q = i - row * per_row;
  const int b = row / keep, k = row - b * keep;
  const int c = q / (P * (P / 8)), r2 = q - c * P * (P / 8);
  const int py = r2 / (P / 8), px = (r2 - py * (P / 8)) * 8;
  const int p = (int)ids[(size_t)b * L + k];
  const int G = W / P;
  const int hy = p / G, hx = p - hy * G;
  const float* src = img + (((size_t)b * C + c) * H + hy * P + py) * W + hx * P + px;
  const f32x4 lo = *reinterpret_cast<const f32x4*>(src), hi = *reinterpret_cast<const f32x4*>(src + 4);
  store8(out + (size_t)row * C * P * P + (c * P + py) * P + px, lo, hi);
}

extern "C" int tmae_patch_gather(const float* imgs, const int64_t* ids_shuffle, void* out, int n, int C, int H, int W,
                                 int patch, int L, int keep, int dtype, void* stream) {
  const long long total = (long long)n * keep * ((C * patch * patch + 7) / 8 * 8);  // padded rows (Kw values)
  if (total == 0) return TMAE_OK;
  if (patch % 8 == 0 && W % 4 == 0 && ((size_t)imgs & 15) == 0 && total / 8 < (1ll << 31)) {
    const dim3 g8((unsigned)((total / 8 + 255) / 256));
    if (dtype == TMAE_BF16)
      hipLaunchKernelGGL(patch_gather8_kernel<bf16>, g8, dim3(256), 0, (hipStream_t)stream, imgs, ids_shuffle,
                         (bf16*)out, n, C, H, W, patch, L, keep);
    else
      hipLaunchKernelGGL(patch_gather8_kernel<float>, g8, dim3(256), 0, (hipStream_t)stream, imgs, ids_shuffle,
                         (float*)out, n, C, H, W, patch, L, keep);
    TMAE_LAUNCH_CHECK("tmae_patch_gather");
  }
  const dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(patch_gather_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, imgs, ids_shuffle, (bf16*)out,
                       n, C, H, W, patch, L, keep);
  else
    hipLaunchKernelGGL(patch_gather_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, imgs, ids_shuffle,
                       (float*)out, n, C, H, W, patch, L, keep);
  TMAE_LAUNCH_CHECK("tmae_patch_gather");
}

// patchify of the reconstruction gradient ("nchpwq -> nhwpqc", MCM.py:497-522): out[b*L + p][(py*P + px)*C + c]
template <typename T>
__global__ void __launch_bounds__(256)
patchify_kernel(const float* __restrict__ img, T* __restrict__ out, int n, int C, int H, int W, int P) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  const int G = W / P, L = (H / P) * G, KP = P * P * C;
  if (i >= (long long)n * L * KP) return;
  const int col = (int)(i % KP);
  const int row = (int)(i / KP);
  const int b = row / L, p = row - b * L;
  const int hy = p / G, hx = p - hy * G;
  const int q = col / C, c = col - q * C;
  const int py = q / P, px = q - py * P;
  out[i] = to_out<T>(img[(((size_t)b * C + c) * H + hy * P + py) * W + hx * P + px]);
}

extern "C" int tmae_patchify(const float* imgs, void* out, int n, int C, int H, int W, int patch, int dtype,
                             void* stream) {
  TMAE_REQUIRE(H % patch == 0 && W % patch == 0, "tmae_patchify: image %dx%d, patch %d", H, W, patch);
  const long long total = (long long)n * C * H * W;
  if (total == 0) return TMAE_OK;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == TMAE_BF16)
    hipLaunchKernelGGL(patchify_kernel<bf16>, grid, dim3(256), 0, (hipStream_t)stream, imgs, (bf16*)out, n, C, H, W,
                       patch);
  else
    hipLaunchKernelGGL(patchify_kernel<float>, grid, dim3(256), 0, (hipStream_t)stream, imgs, (float*)out, n, C, H, W,
                       patch);
  TMAE_LAUNCH_CHECK("tmae_patchify");
}

// decoder_embed backward gather (MCM.py:657-675): token k of image b sat at decoder row
// 0 (k == 0) or 1 + ids_shuffle[b][k-1]; out[b*ntok + k] = dec_grad[b*(L+1) + row] (cast to the operand dtype)
template <typename T>
__global__ void __launch_bounds__(256)
dec_gather_kernel(const float* __restrict__ g, const int64_t* __restrict__ ids, T* __restrict__ out, int n, int ntok,
                  int L, int D) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n * ntok * D) return;
  const int d = (int)(i % D);
  const int r = (int)(i / D);
  const int b = r / ntok, k = r - b * ntok;
  const int row = k == 0 ? 0 : 1 + (int)ids[(size_t)b * L + k - 1];
  out[i] = to_out<T>(g[((size_t)b * (L + 1) + row) * D + d]);
}

// mask_token gradient: sum over every decoder row the mask token filled (MCM.py:660-664)
// per image b, column d: the sum over the masked positions mi in [ntok - 1, L) of the decoder-input gradient row
// 1 + ids[b][mi] (the mask token's gradient, before the fold over images).  Four waves per block split the
// positions round-robin (their loads in flight together) and add their partials in wave order: one serial walk
// over the ~150 positions of an image was a chain of dependent index + row loads (46 us per call).
__global__ void __launch_bounds__(256)
mask_token_bwd_kernel(const float* __restrict__ g, const int64_t* __restrict__ ids, float* __restrict__ part, int n,
                      int ntok, int L, int D) {
  __shared__ float red[4][64];
  __shared__ int rows[256];
  const int b = blockIdx.y;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int d = blockIdx.x * 64 + tx;
  float s = 0.0f;
  // the masked positions' row indexes go through LDS first, so the row loads below are all independent
  for (int c0 = ntok - 1; c0 < L; c0 += 256) {
    const int nc = min(256, L - c0);
    __syncthreads();
    if ((int)threadIdx.x < nc) rows[threadIdx.x] = 1 + (int)ids[(size_t)b * L + c0 + threadIdx.x];
    __syncthreads();
    if (d < D)
      for (int i = ty; i < nc; i += 4) s += g[((size_t)b * (L + 1) + rows[i]) * D + d];
  }
  red[ty][tx] = s;
  __syncthreads();
  if (ty == 0 && d < D) part[(size_t)b * D + d] = ((red[0][tx] + red[1][tx]) + red[2][tx]) + red[3][tx];
}

extern "C" int tmae_decoder_embed_bwd_gather(const float* dec_grad, const int64_t* ids_shuffle, void* tok_grad, int n,
                                             int ntok, int L, int D, int dtype, float* mask_part, float* dmask,
                                             int accumulate, void* stream) {
  TMAE_REQUIRE(dec_grad && ids_shuffle && tok_grad && ntok >= 1 && ntok <= L + 1, "tmae_decoder_embed_bwd_gather: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  const long long total = (long long)n * ntok * D;
  if (total > 0) {
    const dim3 grid((unsigned)((total + 255) / 256));
    if (dtype == TMAE_BF16)
      hipLaunchKernelGGL(dec_gather_kernel<bf16>, grid, dim3(256), 0, st, dec_grad, ids_shuffle, (bf16*)tok_grad, n,
                         ntok, L, D);
    else
      hipLaunchKernelGGL(dec_gather_kernel<float>, grid, dim3(256), 0, st, dec_grad, ids_shuffle, (float*)tok_grad, n,
                         ntok, L, D);
  }
  if (dmask) {
    TMAE_REQUIRE(mask_part != nullptr, "tmae_decoder_embed_bwd_gather: mask_part workspace required");
    hipLaunchKernelGGL(mask_token_bwd_kernel, dim3(ceil_div(D, 64), n), dim3(256), 0, st, dec_grad, ids_shuffle,
                       mask_part, n, ntok, L, D);
    fold_rows(mask_part, n, D, dmask, dmask, D, accumulate, st);
  }
  TMAE_LAUNCH_CHECK("tmae_decoder_embed_bwd_gather");
}

// out = a + b (f32), the out-of-place residual add where autograd keeps the block input
__global__ void __launch_bounds__(256)
add_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ out, long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

extern "C" int tmae_add(const float* a, const float* b, float* out, long long n, void* stream) {
  if (n <= 0) return TMAE_OK;
  hipLaunchKernelGGL(add_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, b, out, n);
  TMAE_LAUNCH_CHECK("tmae_add");
}

// ================================================================== optimizer
// torch.optim.Adam (amsgrad=False) over one flat f32 buffer: g' = g * clip (+ wd * p); m, v moments;
// p -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
__global__ void __launch_bounds__(256)
adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
            long long n, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2_sqrt,
            const float* __restrict__ clip) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float gg = g[i];
  if (clip) gg *= clip[0];
  const float pv = p[i];
  if (wd != 0.0f) gg += wd * pv;
  const float mm = b1 * m[i] + (1.0f - b1) * gg;
  const float vv = b2 * v[i] + (1.0f - b2) * gg * gg;
  m[i] = mm;
  v[i] = vv;
  p[i] = pv - (lr / bc1) * mm / (sqrtf(vv) / bc2_sqrt + eps);
}

extern "C" int tmae_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                         float eps, float weight_decay, int step, const float* clip, void* stream) {
  TMAE_REQUIRE(p && g && m && v && step >= 1, "tmae_adam: bad arguments");
  if (n <= 0) return TMAE_OK;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n,
                     lr, beta1, beta2, eps, weight_decay, (float)bc1, (float)sqrt(bc2), clip);
  TMAE_LAUNCH_CHECK("tmae_adam");
}

// multi-tensor form: table[t] = {p, g, m, v, n, first_chunk, step} (int64; step = address of the tensor's int32
// step count, torch.optim.Adam's per-parameter ``state["step"]``), chunks of 1024 elements; a block finds its
// tensor by binary search over first_chunk.  One launch updates every parameter of a group.  The step counts
// live on the device (advanced by adam_step_kernel right before), so the bias corrections need no host value
// and a captured HIP graph replays a correct optimizer step every time.
// table rows: {p, g, m, v, n, first_chunk, step, bc}; then one int64 per chunk: its row.  The step kernel advances
// each tensor's device step count and writes its bias corrections (f64 pow rounded to f32, as tmae_adam does on
// the host) to bc[0..1] once, instead of every thread of every chunk recomputing two f64 pows.
__global__ void adam_step_kernel(const long long* __restrict__ tab, int nt, float b1, float b2) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nt) return;
  const int step = ++*reinterpret_cast<int*>(tab[8 * t + 6]);
  float* bc = reinterpret_cast<float*>(tab[8 * t + 7]);
  bc[0] = (float)(1.0 - pow((double)b1, (double)step));
  bc[1] = (float)sqrt(1.0 - pow((double)b2, (double)step));
}

__global__ void __launch_bounds__(256)
adam_multi_kernel(const long long* __restrict__ tab, int nt, float lr, float b1, float b2, float eps, float wd,
                  const float* __restrict__ clip) {
  const long long b = blockIdx.x;
  const long long* e = tab + 8 * tab[8 * (long long)nt + b];  // this chunk's row: one load (no search)
  float* __restrict__ p = (float*)e[0];
  const float* __restrict__ g = (const float*)e[1];
  float* __restrict__ m = (float*)e[2];
  float* __restrict__ v = (float*)e[3];
  const long long n = e[4];
  const long long base = (b - e[5]) * 1024 + threadIdx.x;
  const float* bcp = (const float*)e[7];
  const float bc1 = bcp[0], bc2_sqrt = bcp[1];
  const float cs = clip ? clip[0] : 1.0f;
  // a thread's 4 elements 256 apart (each wave access contiguous), every load issued before the math and stores
  float gg[4], pv[4], mv[4], vv[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = base + 256 * u;
    if (i < n) { gg[u] = g[i]; pv[u] = p[i]; mv[u] = m[i]; vv[u] = v[i]; }
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const long long i = base + 256 * u;
    if (i >= n) break;
    float gr = gg[u] * cs;
    if (wd != 0.0f) gr += wd * pv[u];
    const float mm = b1 * mv[u] + (1.0f - b1) * gr;
    const float vq = b2 * vv[u] + (1.0f - b2) * gr * gr;
    m[i] = mm;
    v[i] = vq;
    p[i] = pv[u] - (lr / bc1) * mm / (sqrtf(vq) / bc2_sqrt + eps);
  }
}

extern "C" int tmae_adam_multi(const long long* table, int ntensors, long long nchunks, float lr, float beta1,
                               float beta2, float eps, float weight_decay, const float* clip, void* stream) {
  TMAE_REQUIRE(table && ntensors > 0 && nchunks >= 0, "tmae_adam_multi: bad arguments");
  hipLaunchKernelGGL(adam_step_kernel, dim3((unsigned)((ntensors + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     table, ntensors, beta1, beta2);
  TMAE_LAUNCH_CHECK_NORET("tmae_adam_multi (steps)");
  if (nchunks == 0) return TMAE_OK;
  hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)nchunks), dim3(256), 0, (hipStream_t)stream, table, ntensors,
                     lr, beta1, beta2, eps, weight_decay, clip);
  TMAE_LAUNCH_CHECK("tmae_adam_multi");
}

// clip_grad_norm_(params, max_norm) over a flat gradient buffer: out[0] = ||g||_2 (f64 partials, fixed
// order), out[1] = min(1, max_norm / (norm + 1e-6)) -- the factor applied to the gradients (no host sync)
__global__ void __launch_bounds__(256)
sumsq_partial_kernel(const float* __restrict__ g, long long n, double* __restrict__ part) {
  // 16-B loads, four of them in flight per thread (a 4-B load per iteration ran at ~1.3 TB/s); element
  // assignment and summation order fixed by the grid, so the norm is reproducible
  __shared__ double red[256];
  double s = 0.0;
  const long long n16 = (((unsigned long long)g & 15) == 0) ? n / 16 * 16 : 0;
  const long long stride = (long long)gridDim.x * 256 * 16;
  // block b's window per trip: 4096 elements at b * 4096 (+ stride per trip); thread t: float4s t, t + 256, ...
  for (long long i = (long long)blockIdx.x * 4096 + threadIdx.x * 4; i < n16; i += stride) {
    f32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (i + 1024 * u < n16) ? load4f(g + i + 1024 * u) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += (double)v[u][e] * (double)v[u][e];
  }
  for (long long i = n16 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double x = g[i];
    s += x * x;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256)
clip_final_kernel(const double* __restrict__ part, int np, float max_norm, float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s += part[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float norm = (float)sqrt(red[0]);
    out[0] = norm;
    out[1] = fminf(1.0f, max_norm / (norm + 1e-6f));
  }
}

extern "C" int tmae_grad_norm(const float* g, long long n, double* work, float max_norm, float* out, void* stream) {
  TMAE_REQUIRE(g && work && out, "tmae_grad_norm: null argument");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_partial_kernel, dim3(2048), dim3(256), 0, st, g, n, work);
  hipLaunchKernelGGL(clip_final_kernel, dim3(1), dim3(256), 0, st, work, 2048, max_norm, out);
  TMAE_LAUNCH_CHECK("tmae_grad_norm");
}

// grads *= scale[0] (clip_grad_norm_ applies its factor to the stored gradients)
// 8 elements per thread by 16-B accesses when g is 16-B aligned (one element per thread ran at ~3.8 TB/s)
__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ g, long long n, const float* __restrict__ s) {
  const float f = s[0];
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (((unsigned long long)g & 15) == 0 && i + 8 <= n) {
    f32x4 a, b;
    load8f(g + i, a, b);
    store8(g + i, a * f, b * f);
    return;
  }
  for (long long k = i; k < i + 8 && k < n; ++k) g[k] *= f;
}

extern "C" int tmae_scale(float* g, long long n, const float* scale, void* stream) {
  if (n <= 0) return TMAE_OK;
  hipLaunchKernelGGL(scale_kernel, dim3((unsigned)((n + 2047) / 2048)), dim3(256), 0, (hipStream_t)stream, g, n, scale);
  TMAE_LAUNCH_CHECK("tmae_scale");
}
