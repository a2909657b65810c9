// Weight-gradient ("TN") GEMM for gfx950: out[m][n] = sum_k A(k, m) * B(k, n), both operands stored
// k-major (row k of each is a contiguous run of columns).  This is the contraction of every wgrad of
// the training step: dW[n_out][k_in] = sum_rows dY[row][n_out] * X[row][k_in] (nn.Linear, 1x1 convs)
// and dW[co][tap][ci] = sum_pix dY[pix][co] * X[shift(pix, tap)][ci] (3x3 convs, implicit im2col).
// Both operands are read exactly as the forward produced them (token rows / NHWC maps): no transpose
// pass over HBM.
//
// bf16: the two k x column slabs go global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction) as [k][column] images, and the MFMA fragments (8 consecutive k of one column)
// come out of them with ds_read_b64_tr_b16 (cdna_hip_programming.md T10): two 4-row transposed reads
// per 16x16x32 operand.  32-byte unit u of LDS row r is stored at u ^ f(r), f(r) = (r&3) | ((r>>3)&1)<<2,
// so the 8 rows {0-3, 8-11} (+4) one 32-lane half reads land on 8 distinct bank octets.
// f32 (parity path): register staging with the transposed write into the [column][k] image of the
// NT core, consumed by its exact-f32 16x16x4 MFMA step.
//
// Split-K: the k range is cut into `splits` chunks (grid.y); each workgroup writes its partial tile to
// a f32 workspace [split][M][N]; tmae_tn_reduce sums the splits in a fixed order (bitwise reproducible)
// and scatters into the parameter's own layout.
#pragma once

#include "gemm_core.h"

// ------------------------------------------------------------------ k-major sources
// dense: row k of the operand = source row (k / G) * Gs + off + (k % G), `cols` valid columns
template <typename T> struct KDenseSrc {
  const T* p;
  int ld, cols, G, Gs, off;
  long long sb = 0;  // element offset of problem z (batched launches: blockIdx.z)
  __device__ void batch(int z) { p += z * sb; }
  __device__ const void* addr(int k, int c) const {
    if (c >= cols) return g_tmae_zero_page;
    const int sk = (k / G) * Gs + off + (k % G);
    return p + (size_t)sk * ld + c;
  }
  // row k inside the operand (the caller's K-step lies wholly inside the k range): columns past `cols`
  // read the last 8 columns (their products reach only output rows / columns the epilogue drops);
  // `grouped` (wave-uniform, G < K): the row group k / G is a float-reciprocal quotient with one correction
  // instead of an integer division; ungrouped rows are plain 32-bit offset arithmetic
  __device__ const void* addr_in(int k, int c, float inv_g, bool grouped) const {
    c = min(c, cols - 8);
    int sk = off + k;
    if (grouped) {
      int q = (int)((float)k * inv_g);
      int r = k - q * G;
      if (r >= G) { ++q; r -= G; }
      if (r < 0) { --q; r += G; }
      sk = q * Gs + off + r;
    }
    return p + ((unsigned)sk * (unsigned)ld + (unsigned)c);
  }
};

// implicit im2col of a 3x3 conv (padding 1, stride s) over NHWC maps: row k = output pixel
// (b, oy, ox), column c = tap * Cin + ci; channels [0, c1) from x1, the rest from x2
template <typename T> struct KConvSrc {
  const T* x1;
  const T* x2;
  int c1, ld1, ld2, Cin, H, W, Ho, Wo, stride, cols;
  long long sb1 = 0, sb2 = 0;  // element offsets of problem z's x1 / x2 (batched launches)
  __device__ void batch(int z) {
    x1 += z * sb1;
    if (x2) x2 += z * sb2;
  }
  __device__ const void* addr(int k, int c) const {
    if (c >= cols) return g_tmae_zero_page;
    const int tap = c / Cin, ci = c - tap * Cin;
    const int hw = Ho * Wo;
    const int b = k / hw, rem = k - b * hw;
    const int oy = rem / Wo, ox = rem - oy * Wo;
    const int ky = (tap * 11) >> 5;  // tap / 3
    const int iy = oy * stride - 1 + ky, ix = ox * stride - 1 + (tap - 3 * ky);
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) return g_tmae_zero_page;
    const size_t pix = (size_t)b * H * W + iy * W + ix;
    return ci < c1 ? (const void*)(x1 + pix * ld1 + ci) : (const void*)(x2 + pix * ld2 + (ci - c1));
  }
  // K iterator for the LDS-DMA ring (k = output pixel, issued once per K-step and in order): a lane's column --
  // its tap, channel and source map -- is fixed for the whole launch, and its pixel (b, oy, ox) moves by the
  // K-step's pixel count without the two integer divisions addr() pays per piece per step (~60 VALU: the wgrad
  // K loops were VALU-bound).  Same addresses as addr().
  struct Step { int db, dy, dx; };
  __device__ Step step(int dk) const {
    const int hw = Ho * Wo, r = dk % hw;
    return Step{dk / hw, r / Wo, r % Wo};
  }
  struct It { const T* base; int ldx, k, b, oy, ox, ky, kx; bool col; };
  __device__ It iter(int k, int c) const {
    It it;
    it.col = c < cols;
    const int cc = it.col ? c : 0;
    const int tap = cc / Cin, ci = cc - tap * Cin;
    it.ky = (tap * 11) >> 5;  // tap / 3
    it.kx = tap - 3 * it.ky;
    it.base = ci < c1 ? x1 + ci : x2 + (ci - c1);
    it.ldx = ci < c1 ? ld1 : ld2;
    it.k = k;
    const int hw = Ho * Wo;
    it.b = k / hw;
    const int rem = k - it.b * hw;
    it.oy = rem / Wo;
    it.ox = rem - it.oy * Wo;
    return it;
  }
  // this step's address (the zero page past k1, outside the map or past the columns), then one K-step on
  __device__ const void* next(It& it, int k1, int dk, const Step& st) const {
    const int iy = it.oy * stride - 1 + it.ky, ix = it.ox * stride - 1 + it.kx;
    const bool ok = it.col && it.k < k1 && iy >= 0 && iy < H && ix >= 0 && ix < W;
    const size_t pix = (size_t)it.b * H * W + iy * W + ix;
    const void* a = ok ? (const void*)(it.base + pix * it.ldx) : (const void*)g_tmae_zero_page;
    it.k += dk;
    it.ox += st.dx;
    if (it.ox >= Wo) { it.ox -= Wo; ++it.oy; }
    it.oy += st.dy;
    if (it.oy >= Ho) { it.oy -= Ho; ++it.b; }
    it.b += st.db;
    return a;
  }
};

template <class S, class = void> struct HasKIter : std::false_type {};
template <class S>
struct HasKIter<S, std::void_t<typename S::It>> : std::true_type {};
template <class S, bool B> struct KItOf { struct type {}; };
template <class S> struct KItOf<S, true> { using type = typename S::It; };
template <class S, bool B> struct KStepOf { struct type {}; };
template <class S> struct KStepOf<S, true> { using type = typename S::Step; };

// partial tile -> workspace slab of this split; bws (optional): the bias slab [split][M] of column sums
struct EpiSplitWs {
  float* ws;
  int N;
  long long slab;
  float* bws;
  int M;
  __device__ void batch(int, int) {}
  __device__ void operator()(int m, int n, f32x4 v) const { store4(ws + (size_t)m * N + n, v); }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi) const { store8(ws + (size_t)m * N + n, lo, hi); }
};

// in-range address of a k-major source: KDenseSrc's addr_in, the checked addr for the others
template <class S> __device__ __forceinline__ float tn_inv_g(const S&) { return 0.0f; }
template <typename T> __device__ __forceinline__ float tn_inv_g(const KDenseSrc<T>& s) { return 1.0f / (float)s.G; }
template <class S> __device__ __forceinline__ bool tn_grouped(const S&, int) { return true; }
template <typename T> __device__ __forceinline__ bool tn_grouped(const KDenseSrc<T>& s, int K) { return s.G < K; }
template <class S> __device__ __forceinline__ const void* tn_addr_in(const S& s, int k, int c, float, bool) {
  return s.addr(k, c);
}
template <typename T>
__device__ __forceinline__ const void* tn_addr_in(const KDenseSrc<T>& s, int k, int c, float inv_g, bool grouped) {
  return s.addr_in(k, c, inv_g, grouped);
}

__device__ __forceinline__ int tn_swz(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

typedef __attribute__((ext_vector_type(4))) short tn_s4;
typedef __attribute__((address_space(3))) tn_s4 tn_lds_s4;

__device__ __forceinline__ bf16x8 tn_frag(const unsigned char* img, int rb, int r1, int u, int p) {
  const int r2 = r1 + 4;
  const tn_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (tn_lds_s4*)(img + r1 * rb + 32 * (u ^ tn_swz(r1)) + 8 * p));
  const tn_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (tn_lds_s4*)(img + r2 * rb + 32 * (u ^ tn_swz(r2)) + 8 * p));
  typedef __attribute__((ext_vector_type(8))) short s8;
  s8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return *reinterpret_cast<bf16x8*>(&v);
}

// ------------------------------------------------------------------ bf16 kernel
// AS = M-side source (MFMA B operand), BS = N-side source (MFMA A operand, rows of the accumulator).
// BIAS: also the column sums sum_k A(k, m) of this split's k range (the bias gradient of the layer whose
// output gradient A is, reference: the colsum over rows of dY) by MFMAs against an all-ones A fragment:
// ones^T B = the column sums in every accumulator row.  The same sums are wanted by every (tn, wn) that
// shares the M columns, so fragment j of a wave is computed by exactly one of them (j = r mod P, P =
// ntn * WGN sharers): at most ceil(TM / P) extra MFMAs per K-substep on top of TN * TM.
template <int BN, int BM, int WGN, int NW, bool BIAS, class AS, class BS>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 1 : 2)
gemm_tn_bf16_kernel(AS as, BS bs, EpiSplitWs epi, int M, int N, int K, int kchunk) {
  constexpr int BK = 64;
  constexpr int WGM = NW / WGN;
  constexpr int WN = BN / WGN, WM = BM / WGM;
  constexpr int TN = WN / 16, TM = WM / 16;
  constexpr int RBN = BN * 2, RBM = BM * 2;
  constexpr int IMG_N = BK * RBN, IMG_M = BK * RBM;
  constexpr int STAGE = IMG_N + IMG_M;
  constexpr int WPN = IMG_N / 1024 / NW, WPM = IMG_M / 1024 / NW;
  static_assert(RBN >= 256 && RBM >= 256, "tn: LDS rows of at least 8 bank octets");
  static_assert(WPN * NW * 1024 == IMG_N && WPM * NW * 1024 == IMG_M, "tn: pieces per wave");
  static_assert(TN >= 1 && TM >= 1, "tn: tile");
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * STAGE / 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  int tn, tm;
  tile_order(xcd_remap(blockIdx.x, gridDim.x), ntn, ntm, tn, tm);
  const int k0 = blockIdx.y * kchunk, k1 = min(K, k0 + kchunk);
  const int nk = k1 > k0 ? (k1 - k0 + BK - 1) / BK : 0;
  // problem z of a batched launch: its sources, its [splits] slabs and its bias slab
  as.batch(blockIdx.z);
  bs.batch(blockIdx.z);
  epi.ws += ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * epi.slab;
  if (epi.bws) epi.bws += (size_t)blockIdx.z * gridDim.y * M;
  // bias fragments owned by this wave (wave-uniform): j with j % P == r % P
  const int bias_P = ntn * WGN, bias_r = tn * WGN + wn;

  // this lane's DMA slots: piece p of the wave covers image bytes [(wave + NW p) KiB, +1 KiB)
  int nrow[WPN], ncol[WPN], mrow[WPM], mcol[WPM];
#pragma unroll
  for (int p = 0; p < WPN; ++p) {
    const int byte = (wave + NW * p) * 1024 + 16 * lane;
    const int r = byte / RBN, pc = (byte % RBN) / 16;
    nrow[p] = r;
    ncol[p] = tn * BN + 8 * (2 * ((pc >> 1) ^ tn_swz(r)) + (pc & 1));
  }
#pragma unroll
  for (int p = 0; p < WPM; ++p) {
    const int byte = (wave + NW * p) * 1024 + 16 * lane;
    const int r = byte / RBM, pc = (byte % RBM) / 16;
    mrow[p] = r;
    mcol[p] = tm * BM + 8 * (2 * ((pc >> 1) ^ tn_swz(r)) + (pc & 1));
  }
  const unsigned wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)lds;
  const float inv_ga = tn_inv_g(as), inv_gb = tn_inv_g(bs);
  const bool grp_a = tn_grouped(as, K), grp_b = tn_grouped(bs, K);  // wave-uniform
  // N-side K iterators (the implicit im2col source): issue() below runs once per K-step, in order from step 0
  constexpr bool BIT = HasKIter<BS>::value;
  typename KItOf<BS, BIT>::type bit[WPN];
  typename KStepOf<BS, BIT>::type bst{};
  if constexpr (BIT) {
    bst = bs.step(BK);
#pragma unroll
    for (int p = 0; p < WPN; ++p) bit[p] = bs.iter(k0 + nrow[p], ncol[p]);
  }
  auto issue = [&](int stage, int kt) {
    const unsigned sb = lds_base + (unsigned)stage * STAGE;
    const int kb = k0 + kt * BK;
    if constexpr (BIT) {
      const bool full = kb + BK <= k1;
#pragma unroll
      for (int p = 0; p < WPN; ++p) glds16(bs.next(bit[p], k1, BK, bst), sb + (wave_u + NW * p) * 1024u);
      if (full) {
#pragma unroll
        for (int p = 0; p < WPM; ++p)
          glds16(tn_addr_in(as, kb + mrow[p], mcol[p], inv_ga, grp_a), sb + IMG_N + (wave_u + NW * p) * 1024u);
      } else {
#pragma unroll
        for (int p = 0; p < WPM; ++p) {
          const int k = kb + mrow[p];
          glds16(k < k1 ? as.addr(k, mcol[p]) : (const void*)g_tmae_zero_page, sb + IMG_N + (wave_u + NW * p) * 1024u);
        }
      }
      return;
    }
    if (kb + BK <= k1) {  // whole K-step inside this split's range (wave-uniform): no per-row bounds select
#pragma unroll
      for (int p = 0; p < WPN; ++p) glds16(tn_addr_in(bs, kb + nrow[p], ncol[p], inv_gb, grp_b), sb + (wave_u + NW * p) * 1024u);
#pragma unroll
      for (int p = 0; p < WPM; ++p)
        glds16(tn_addr_in(as, kb + mrow[p], mcol[p], inv_ga, grp_a), sb + IMG_N + (wave_u + NW * p) * 1024u);
      return;
    }
#pragma unroll
    for (int p = 0; p < WPN; ++p) {
      const int k = kb + nrow[p];
      glds16(k < k1 ? bs.addr(k, ncol[p]) : (const void*)g_tmae_zero_page, sb + (wave_u + NW * p) * 1024u);
    }
#pragma unroll
    for (int p = 0; p < WPM; ++p) {
      const int k = kb + mrow[p];
      glds16(k < k1 ? as.addr(k, mcol[p]) : (const void*)g_tmae_zero_page, sb + IMG_N + (wave_u + NW * p) * 1024u);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  f32x4 bacc[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) bacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.0f;

  const int g = lane >> 4, ii = lane & 15, q = ii >> 2, pp = ii & 3;
  if (nk > 0) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) issue(stage ^ 1, kt + 1);
      const unsigned char* base = reinterpret_cast<const unsigned char*>(lds) + stage * STAGE;
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        const int r1 = 32 * s + 8 * g + q;
        bf16x8 a[TN], b[TM];
#pragma unroll
        for (int i = 0; i < TN; ++i) a[i] = tn_frag(base, RBN, r1, (wn * WN + 16 * i) >> 4, pp);
#pragma unroll
        for (int j = 0; j < TM; ++j) b[j] = tn_frag(base + IMG_N, RBM, r1, (wm * WM + 16 * j) >> 4, pp);
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        if constexpr (BIAS) {
#pragma unroll
          for (int j = 0; j < TM; ++j)
            if ((j - bias_r) % bias_P == 0) bacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, b[j], bacc[j], 0, 0, 0);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stage ^= 1;
    }
  }
  if constexpr (BIAS) {
    // every accumulator row holds the column sums: lanes 0-15 (rows 0-3, column fr) store them
    float* bw = epi.bws + (size_t)blockIdx.y * M;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = tm * BM + wm * WM + 16 * j + ii;
      if ((j - bias_r) % bias_P == 0 && lane < 16 && m < M) bw[m] = bacc[j][0];
    }
  }
  static_assert(NW * EpiRegion<WN>::FLOATS * 4 <= 2 * STAGE, "tn: epilogue region exceeds the LDS ring");
  epilogue_lds<TN, TM, WN>(epi, acc, reinterpret_cast<float*>(lds) + wave * EpiRegion<WN>::FLOATS,
                           tn * BN + wn * WN, tm * BM + wm * WM, lane, M, N);
}

// ------------------------------------------------------------------ f32 kernel (parity path)
// 4 waves, 64 x 64 tile, BK = 32: each thread loads 16-B row chunks of the k-major slabs and writes
// them transposed into the [column][k] image that mfma_tile<float> reads.
template <class AS, class BS>
__global__ void __launch_bounds__(256, 2)
gemm_tn_f32_kernel(AS as, BS bs, EpiSplitWs epi, int M, int N, int K, int kchunk) {
  constexpr int BN = 64, BM = 64, WGN = 2, BK = 32;
  constexpr int WN = BN / WGN, WM = BM / 2, TN = WN / 16, TM = WM / 16;
  constexpr int ROWS = BN + BM;
  __shared__ __attribute__((aligned(16))) uint4 lds[ROWS * 8 + 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  int tn, tm;
  tile_order(xcd_remap(blockIdx.x, gridDim.x), (N + BN - 1) / BN, (M + BM - 1) / BM, tn, tm);
  const int k0 = blockIdx.y * kchunk, k1 = min(K, k0 + kchunk);
  epi.ws += (size_t)blockIdx.y * epi.slab;
  float* fl = reinterpret_cast<float*>(lds);
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per stage: BK rows x (BN + BM) columns = 32 x 128 floats = 1024 chunks of 4: 4 per thread
  for (int kb = k0; kb < k1; kb += BK) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int cidx = tid + 256 * t;  // 0..1023
      const int r = cidx >> 5, c4 = (cidx & 31) * 4;  // k row, column (0..127)
      const int k = kb + r;
      f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
      int lrow;
      if (c4 < BN) {
        lrow = c4;
        if (k < k1) v = *reinterpret_cast<const f32x4*>(bs.addr(k, tn * BN + c4));
      } else {
        lrow = c4;  // BN + (c4 - BN)
        if (k < k1) v = *reinterpret_cast<const f32x4*>(as.addr(k, tm * BM + (c4 - BN)));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = lrow + e;
        fl[(row * 8 + ((r >> 2) ^ ((row >> 1) & 7))) * 4 + (r & 3)] = v[e];
      }
    }
    __syncthreads();
    mfma_tile<float, BN, WN, WM, TN, TM>(lds, wn, wm, lane, acc);
    __syncthreads();
  }
  epilogue_lds<TN, TM, WN>(epi, acc, fl + wave * EpiRegion<WN>::FLOATS, tn * BN + wn * WN, tm * BM + wm * WM, lane,
                           M, N);
}

// ------------------------------------------------------------------ launch
struct TnPlan { int bn, bm, nw, splits, kchunk; };

static inline TnPlan tn_plan(int M, int N, int K, bool bf, int slot_div = 1, int nb = 1) {
  TnPlan p;
  if (!bf) {
    p.bn = 64; p.bm = 64; p.nw = 4;
  } else {
    const long long t256 = (long long)ceil_div(N, 256) * ceil_div(M, 256);
    const double u256 = ((double)N / (ceil_div(N, 256) * 256.0)) * ((double)M / (ceil_div(M, 256) * 256.0));
    if (u256 > 0.7 && t256 * 8 >= 64) { p.bn = 256; p.bm = 256; p.nw = 8; }
    else { p.bn = 128; p.bm = 128; p.nw = 4; }
  }
  const int tiles = ceil_div(N, p.bn) * ceil_div(M, p.bm) * std::max(1, nb);  // nb problems share the slots
  const int slots = (p.nw == 8 ? 256 : 512) / std::max(1, slot_div);
  const int kmin = bf ? 256 : 128;
  // splits: as many as fit ONE round of the slots (floor): with the ceiling, tiles * splits overshot the
  // 256 slots of the 8-wave tile on every encoder weight gradient (qkv 270, fc1 / fc2 288, proj 261
  // workgroups), and the few workgroups of the second round took a whole round of time
  int s = std::max(1, slots / tiles);
  s = std::max(1, std::min(s, std::max(1, K / kmin)));
  s = std::min(s, 64);
  const int step = bf ? 64 : 32;
  p.kchunk = ceil_div(ceil_div(K, s), step) * step;
  p.splits = ceil_div(K, p.kchunk);
  return p;
}

// bws (bias slab [splits][M]) non-null: the kernel also forms the column sums of A (BIAS instantiation)
template <class AS, class BS>
static int launch_tn_bf16(const TnPlan& p, const AS& as, const BS& bs, float* ws, float* bws, int M, int N, int K,
                          hipStream_t st, int nb = 1) {
  const int tiles = ceil_div(N, p.bn) * ceil_div(M, p.bm);
  EpiSplitWs e{ws, N, (long long)M * N, bws, M};
  if (p.nw == 8) {
    if (bws)
      hipLaunchKernelGGL((gemm_tn_bf16_kernel<256, 256, 2, 8, true, AS, BS>), dim3(tiles, p.splits, nb), dim3(512), 0, st,
                         as, bs, e, M, N, K, p.kchunk);
    else
      hipLaunchKernelGGL((gemm_tn_bf16_kernel<256, 256, 2, 8, false, AS, BS>), dim3(tiles, p.splits, nb), dim3(512), 0, st,
                         as, bs, e, M, N, K, p.kchunk);
  } else {
    if (bws)
      hipLaunchKernelGGL((gemm_tn_bf16_kernel<128, 128, 2, 4, true, AS, BS>), dim3(tiles, p.splits, nb), dim3(256), 0, st,
                         as, bs, e, M, N, K, p.kchunk);
    else
      hipLaunchKernelGGL((gemm_tn_bf16_kernel<128, 128, 2, 4, false, AS, BS>), dim3(tiles, p.splits, nb), dim3(256), 0, st,
                         as, bs, e, M, N, K, p.kchunk);
  }
  TMAE_LAUNCH_CHECK("tmae_wgrad");
}

template <class AS, class BS>
static int launch_tn_f32(const TnPlan& p, const AS& as, const BS& bs, float* ws, int M, int N, int K, hipStream_t st) {
  const int tiles = ceil_div(N, 64) * ceil_div(M, 64);
  EpiSplitWs e{ws, N, (long long)M * N, nullptr, M};
  hipLaunchKernelGGL((gemm_tn_f32_kernel<AS, BS>), dim3(tiles, p.splits), dim3(256), 0, st, as, bs, e, M, N, K,
                     p.kchunk);
  TMAE_LAUNCH_CHECK("tmae_wgrad");
}
