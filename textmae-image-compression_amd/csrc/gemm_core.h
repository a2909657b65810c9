// MFMA GEMM core for gfx950 shared by gemm.hip (token GEMMs) and conv.hip (LIC convs).
//
//   out[m][n] = epilogue( sum_k X[m][k] * W[n][k] + bias[n] )     for every problem of a batch
//
// W is a [N][K] row-major weight in the operand type T (nn.Linear layout; conv weights re-laid out
// to [Cout][ky][kx][Cin] at weight-prep time).  X rows come from a row source: dense token rows,
// an implicit-GEMM 3x3 conv gather over NHWC maps, or the patch-embed gather over the image.
//
// Two staging variants of the same tile/LDS/MFMA design:
//   gemm_glds_kernel: global -> LDS with global_load_lds_dwordx4 (no VGPR round trip, 16 B/lane),
//                     the per-lane SOURCE address carries the LDS swizzle, masked lanes read a zero
//                     page; 2-stage LDS ring, next tile in flight under the current tile's MFMAs.
//   gemm_reg_kernel:  global -> VGPR -> LDS, for sources that must be converted on the way (the
//                     f32 image into bf16 patch-embed operands).
// LDS rows are 128 B (64 bf16 / 32 f32 of K); 16-B chunk c of row r sits at c ^ ((r >> 1) & 7), which
// makes the ds_read_b128 fragment reads of 16 consecutive rows conflict-free.  The MFMA is issued
// swapped (A = weight rows, B = activation rows) so every lane owns 4 consecutive output columns.
//   bf16: v_mfma_f32_16x16x32_bf16 (f32 accumulate)       f32: v_mfma_f32_16x16x4_f32 (exact f32)
#pragma once

#include <stdlib.h>

#include <algorithm>
#include <cmath>
#include <type_traits>
#include <utility>

#include "common.h"

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// zero page for masked glds lanes (one copy per translation unit; no relocatable device code)
static __device__ __attribute__((aligned(64))) uint4 g_tmae_zero_page[4] = {};

// One LDS-DMA piece: 64 lanes x 16 B -> LDS [lds_addr, lds_addr + 1 KiB), lane-linear.  Issued from
// inline asm so hipcc does not count it: with the builtin, hipcc cannot prove that the stage being
// filled does not alias the stage being read and puts an s_waitcnt vmcnt(0) in front of the next
// ds_read, serialising every K-step behind its own prefetch.  The caller waits (vmcnt) itself.
// M0 is saved/restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_addr) {
  unsigned keep;
  lds_addr = __builtin_amdgcn_readfirstlane(lds_addr);  // wave-uniform by construction; pin it to an SGPR
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_addr)
               : "memory");
}

template <typename T> struct Elt;
template <> struct Elt<bf16> { static constexpr int EPC = 8; };
template <> struct Elt<float> { static constexpr int EPC = 4; };

// batch decomposition: problem b = b1 * n2 + b2 -> element offset b1 * s1 + b2 * s2
struct BStride {
  long long s1, s2;
  __device__ __forceinline__ long long at(int b1, int b2) const { return (long long)b1 * s1 + (long long)b2 * s2; }
};

template <typename T> __device__ __forceinline__ uint4 load_chunk_from_f32(const float* p);
template <> __device__ __forceinline__ uint4 load_chunk_from_f32<float>(const float* p) {
  return *reinterpret_cast<const uint4*>(p);
}
template <> __device__ __forceinline__ uint4 load_chunk_from_f32<bf16>(const float* p) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  return pack8_bf16(a, b);
}

// ------------------------------------------------------------------ row sources
// Dense rows of T.  source row = (m / G) * Gs + off + (m % G)   (strided views: drop cls rows)
template <typename T> struct DenseSrc {
  const T* p;
  int ld, rows, K, G, Gs, off;
  BStride bs;
  struct Row { const T* ptr; };
  __device__ void batch(int b1, int b2) { p += bs.at(b1, b2); }
  // rows past the end are clamped to the last row: their products only reach output rows / columns that
  // every epilogue drops (m < M, n < N), so no lane needs a zero-page select in the K loop
  __device__ Row row(int m) const {
    if (rows <= 0) return {nullptr};
    m = min(m, rows - 1);
    // ungrouped sources (G >= rows: every weight, most token matrices; wave-uniform) skip the integer division,
    // ~40 VALU instructions per DMA row in every workgroup's prologue
    const int sm = G >= rows ? off + m : (m / G) * Gs + off + (m % G);
    return {p + (size_t)sm * ld};
  }
  __device__ const void* addr_k(const Row& r, int k) const {
    return (r.ptr && k < K) ? (const void*)(r.ptr + k) : (const void*)g_tmae_zero_page;
  }
  __device__ const void* addr(const Row& r, int kt, int c) const {
    return addr_k(r, kt * 8 * Elt<T>::EPC + c * Elt<T>::EPC);
  }
  // a K-step that lies wholly inside K (the caller checks that, wave-uniformly): plain pointer arithmetic
  __device__ const void* addr_full(const Row& r, int kt, int c) const {
    return r.ptr + kt * 8 * Elt<T>::EPC + c * Elt<T>::EPC;
  }
  __device__ uint4 load(const Row& r, int kt, int c) const { return *reinterpret_cast<const uint4*>(addr(r, kt, c)); }
};

// Implicit-GEMM 3x3 conv (padding 1, stride s) over NHWC maps of T; input channels [0,c1) from x1,
// [c1, c1+c2) from x2 (torch.cat without a copy, MCM.py:761,766,780).  K = (ky*3 + kx) * Cin + c.
template <typename T> struct ConvSrc {
  const T* x1;
  const T* x2;
  int c1, ld1, ld2, Cin, H, W, Ho, Wo, stride, rows, K;
  float inv_cin;
  BStride bs1, bs2;
  struct Row { int pix; int iy0; int ix0; bool ok; };
  __device__ void batch(int b1, int b2) { x1 += bs1.at(b1, b2); x2 += bs2.at(b1, b2); }
  __device__ Row row(int m) const {
    if (m >= rows) return {0, 0, 0, false};
    const int hw = Ho * Wo;
    const int b = m / hw, rem = m - b * hw;
    const int oy = rem / Wo, ox = rem - oy * Wo;
    return {b * H * W, oy * stride - 1, ox * stride - 1, true};
  }
  __device__ const void* addr(const Row& r, int kt, int c) const {
    return addr_k(r, kt * 8 * Elt<T>::EPC + c * Elt<T>::EPC);
  }
  __device__ const void* addr_k(const Row& r, int k) const {
    if (!r.ok || k >= K) return g_tmae_zero_page;
    int tap = (int)((float)k * inv_cin);
    if (tap * Cin > k) --tap;
    if ((tap + 1) * Cin <= k) ++tap;
    const int ci = k - tap * Cin;
    const int ky = (tap * 11) >> 5;  // tap / 3 for tap < 9
    const int iy = r.iy0 + ky, ix = r.ix0 + (tap - 3 * ky);
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) return g_tmae_zero_page;
    const int pix = r.pix + iy * W + ix;
    return (ci < c1) ? (const void*)(x1 + (size_t)pix * ld1 + ci) : (const void*)(x2 + (size_t)pix * ld2 + (ci - c1));
  }
  __device__ uint4 load(const Row& r, int kt, int c) const { return *reinterpret_cast<const uint4*>(addr(r, kt, c)); }
};

// ConvSrc with a K iterator for the LDS-DMA ring, whose K-steps are issued once each and in order from step 0.
// tmae_conv3x3 picks it for bf16 inputs of >= 128 channels.  With 64 channels a chunk changes tap every K-step,
// and the pointer rebuild costs more than addr_k's division: VGG's 64-channel layers ran 6 % slower with the
// iterator.  A kernel that has both paths is slower on either, so they are separate instantiations.
template <typename T> struct ConvSrcIt : ConvSrc<T> {
  using ConvSrc<T>::x1; using ConvSrc<T>::x2; using ConvSrc<T>::c1; using ConvSrc<T>::ld1; using ConvSrc<T>::ld2;
  using ConvSrc<T>::Cin; using ConvSrc<T>::H; using ConvSrc<T>::W;
  using Row = typename ConvSrc<T>::Row;
  // K iterator for the LDS-DMA ring, whose K-steps are issued once each and in order from step 0: a lane's chunk
  // carries its tap and channel from step to step (one add and a compare; the tap's pixel pointers are rebuilt
  // only when the chunk crosses into the next tap, every Cin / 64 steps) instead of dividing them out of k per
  // step (~35 VALU per chunk, which made these GEMMs 30-50 % slower than a dense GEMM of the same shape).  The
  // addresses are exactly addr_k's.
  struct It { const T* p1; const T* p2; int ci, tap, pix, iy0, ix0; bool ok, in; };
  __device__ void it_tap(It& it) const {
    const int ky = (it.tap * 11) >> 5, kx = it.tap - 3 * ky;  // tap / 3 for tap < 9
    const int iy = it.iy0 + ky, ix = it.ix0 + kx;
    it.in = it.ok && it.tap < 9 && iy >= 0 && iy < H && ix >= 0 && ix < W;
    const int pix = it.in ? it.pix + iy * W + ix : 0;
    it.p1 = x1 + (size_t)pix * ld1;
    it.p2 = x2 ? x2 + (size_t)pix * ld2 - c1 : it.p1;
  }
  __device__ It iter(const Row& r, int c) const {
    It it{nullptr, nullptr, c * Elt<T>::EPC, 0, r.pix, r.iy0, r.ix0, r.ok && Cin > 0, false};
    while (it.ok && it.ci >= Cin) { it.ci -= Cin; ++it.tap; }
    it_tap(it);
    return it;
  }
  // this step's chunk address, then the iterator moves one K-step on
  __device__ const void* next(It& it) const {
    const void* a = !it.in ? (const void*)g_tmae_zero_page
                           : it.ci < c1 ? (const void*)(it.p1 + it.ci) : (const void*)(it.p2 + it.ci);
    it.ci += 8 * Elt<T>::EPC;
    if (it.ci >= Cin && it.ok) {
      do { it.ci -= Cin; ++it.tap; } while (it.ci >= Cin);
      it_tap(it);
    }
    return a;
  }
};

template <class S, class = void> struct HasIter : std::false_type {};
template <class S>
struct HasIter<S, std::void_t<typename S::It>> : std::true_type {};
template <class S, bool B> struct ItOf { using type = int; };
template <class S> struct ItOf<S, true> { using type = typename S::It; };

// Patch-embed gather over the KEPT patches (timm PatchEmbed conv16/s16 as a GEMM, MCM.py:615):
// row m = (image b, kept rank k) reads patch ids_shuffle[b][k] of the f32 NCHW image; converts.
template <typename T> struct PatchSrc {
  const float* img;
  const int64_t* ids;
  int L, keep, C, H, W, P, G, rows, K;
  struct Row { const float* base; };
  __device__ void batch(int, int) {}
  __device__ Row row(int m) const {
    if (m >= rows) return {nullptr};
    const int b = m / keep, k = m - b * keep;
    const int p = (int)ids[(size_t)b * L + k];
    const int hy = p / G, hx = p - hy * G;
    return {img + (size_t)b * C * H * W + (size_t)(hy * P) * W + hx * P};
  }
  __device__ uint4 load(const Row& r, int kt, int c) const {
    constexpr int EPC = Elt<T>::EPC;
    const int k = kt * 8 * EPC + c * EPC;
    if (!r.base || k >= K) return uint4{0, 0, 0, 0};
    const int pp = P * P;
    if (P % EPC == 0) {  // a chunk is EPC pixels of one patch row
      const int ch = k / pp, rem = k - ch * pp;
      const int py = rem / P, px = rem - py * P;
      return load_chunk_from_f32<T>(r.base + (ch * H + py) * W + px);
    }
    // patch rows that are not whole chunks (ViT-H: 14 pixels): element by element, zero past K
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kk = k + e;
      const int ch = kk / pp, rem = kk - ch * pp;
      const int py = rem / P, px = rem - py * P;
      v[e] = (e < EPC && kk < K) ? r.base[(ch * H + py) * W + px] : 0.0f;
    }
    const f32x4 a{v[0], v[1], v[2], v[3]}, b{v[4], v[5], v[6], v[7]};
    if constexpr (sizeof(T) == 2) return pack8_bf16(a, b);
    else return *reinterpret_cast<const uint4*>(&a);
  }
};

// address of a whole (in-K) K-step chunk: the source's addr_full when it has one, else its checked addr
template <class S, class = void> struct HasAddrFull : std::false_type {};
template <class S>
struct HasAddrFull<S, std::void_t<decltype(std::declval<const S&>().addr_full(std::declval<const typename S::Row&>(), 0, 0))>>
    : std::true_type {};
template <class S>
__device__ __forceinline__ const void* src_addr_full(const S& s, const typename S::Row& r, int kt, int c) {
  if constexpr (HasAddrFull<S>::value) return s.addr_full(r, kt, c);
  else return s.addr(r, kt, c);
}

// ------------------------------------------------------------------ tile order
// logical tile id -> (n tile, m tile): groups of 8 M-tiles x all N-tiles, M fastest, so workgroups
// running together share a few activation panels and weight panels in L2.
__device__ __forceinline__ void tile_order(int t, int ntn, int ntm, int& tn, int& tm) {
  constexpr int GM = 8;
  const int group = GM * ntn;
  const int first_m = (t / group) * GM;
  const int gm = min(ntm - first_m, GM);
  const int r = t - (t / group) * group;
  tm = first_m + r % gm;
  tn = r / gm;
}

// ------------------------------------------------------------------ shared compute step
template <typename T, int BN, int WN, int WM, int TN, int TM>
__device__ __forceinline__ void mfma_tile(const uint4* base, int wn, int wm, int lane, f32x4 (&acc)[TN][TM]) {
  const int fr = lane & 15, fq = lane >> 4;
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
}

// ------------------------------------------------------------------ epilogue
// In the MFMA layout a lane holds 4 consecutive output columns of one row per 16x16 block, so
// direct stores write 16 rows x 32 B per instruction: measured 0.9-1.4 TB/s, the epilogue took ~40 %
// of a K=768 GEMM.  Instead each wave transposes its accumulators through its own LDS region
// (16 rows x WN columns of f32 at a time, rows padded by 16 B: conflict-free ds_write_b128) and
// every lane then emits 8 CONSECUTIVE columns of one row: per instruction WN/8 lanes cover a row
// segment of WN columns (full 128-256 B lines for bf16 out).
//
// Functors provide operator()(m, n, f32x4) for 4 columns and optionally wide(m, n, lo, hi) for 8.
//
// The epilogue's own global loads must not wait behind its stores: gfx9 counts loads and stores in
// one in-order vmcnt, so a load issued after a store and then waited for (s_waitcnt vmcnt(0)) waits
// for that store's completion too.  Loaded inline per 8-column emit, every bias / residual load exposed
// a full store round trip (the 256 x 256 fc1 epilogue ran at 2 TB/s).  Two optional hooks let the
// epilogue issue them ahead of the stores instead:
//   prefetch(n, N)     per-lane column data (bias of this lane's 8 columns; the column of a lane is
//                      fixed for the whole epilogue), loaded once into the functor's local copy;
//   fetch(m, n) -> Pre per-(row, 8 columns) operands (residual, addend), issued one 16-row block ahead
//                      and consumed by wide(m, n, lo, hi, pre).
template <class E, class = void> struct HasWide : std::false_type {};
template <class E>
struct HasWide<E, std::void_t<decltype(std::declval<const E&>().wide(0, 0, f32x4{}, f32x4{}))>> : std::true_type {};
template <class E, class = void> struct HasPrefetch : std::false_type {};
template <class E>
struct HasPrefetch<E, std::void_t<decltype(std::declval<E&>().prefetch(0, 0))>> : std::true_type {};
template <class E, class = void> struct HasFetch : std::false_type {};
template <class E>
struct HasFetch<E, std::void_t<decltype(std::declval<const E&>().fetch(0, 0))>> : std::true_type {};

template <class EPI>
__device__ __forceinline__ void epi_emit8(const EPI& epi, int m, int n, f32x4 lo, f32x4 hi, int N) {
  if constexpr (HasWide<EPI>::value) {
    if (n + 8 <= N) {
      epi.wide(m, n, lo, hi);
      return;
    }
  }
  if (n < N) epi(m, n, lo);
  if (n + 4 < N) epi(m, n + 4, hi);
}

// the functor copy one lane's epilogue runs on (column data prefetched)
template <class EPI> __device__ __forceinline__ EPI epi_for_lane(const EPI& epi, int n, int N) {
  EPI e = epi;
  if constexpr (HasPrefetch<EPI>::value) e.prefetch(n, N);
  return e;
}

template <class EPI> struct EpiPre { struct None {}; };
template <class EPI, bool F = HasFetch<EPI>::value> struct PreOf { using type = typename EpiPre<EPI>::None; };
template <class EPI> struct PreOf<EPI, true> { using type = decltype(std::declval<const EPI&>().fetch(0, 0)); };

template <class EPI>
__device__ __forceinline__ void epi_fetch(const EPI& e, int m, int n, int M, int N, typename PreOf<EPI>::type& p) {
  if constexpr (HasFetch<EPI>::value) {
    if (m < M && n + 8 <= N) p = e.fetch(m, n);
  }
}

// emit with a fetched operand set (wide path) or the plain 4-column path at the N tail
template <class EPI>
__device__ __forceinline__ void epi_emit8_pre(const EPI& e, int m, int n, f32x4 lo, f32x4 hi, int N,
                                              const typename PreOf<EPI>::type& p) {
  if constexpr (HasFetch<EPI>::value) {
    if (n + 8 <= N) {
      e.wide(m, n, lo, hi, p);
      return;
    }
    if (n < N) e(m, n, lo);
    if (n + 4 < N) e(m, n + 4, hi);
  } else {
    epi_emit8(e, m, n, lo, hi, N);
  }
}

#ifndef TMAE_EPI_BF16_DIRECT
#define TMAE_EPI_BF16_DIRECT 1  // A/B builds: 0 = plain bf16 stores through the f32 transpose (epilogue_lds)
#endif
#ifndef TMAE_EPI_DEEP_ALWAYS
#define TMAE_EPI_DEEP_ALWAYS 0  // A/B builds: 1 = the one-block-ahead fetch for every instantiation
#endif

template <int WN> struct EpiRegion {
  static constexpr int ST = WN + 4;          // row stride (floats)
  static constexpr int FLOATS = 16 * ST;     // one wave's region
};

// acc[i][j]: rows n = 16 i + 4 fq + r of D (weight side), column m = 16 j + fr (activation side)
template <int TN, int TM, int WN, class EPI>
__device__ __forceinline__ void epilogue_lds(const EPI& epi, const f32x4 (&acc)[TN][TM], float* region, int n0,
                                             int m0, int lane, int M, int N) {
  static_assert(WN >= 32 && WN % 32 == 0, "epilogue_lds: WN must be a multiple of 32");
  constexpr int ST = EpiRegion<WN>::ST;
  constexpr int LPR = WN / 8;   // lanes per row
  constexpr int RPI = 64 / LPR; // rows per read round
  constexpr int QR = 16 / RPI;  // read rounds per 16-row block
  const int fr = lane & 15, fq = lane >> 4;
  const int rr = lane / LPR, cc = lane - rr * LPR;
  const int ncol = n0 + 8 * cc;
  const EPI e = epi_for_lane(epi, ncol, N);
  using Pre = typename PreOf<EPI>::type;
  // Fetch depth: one block ahead (two operand sets live) unless those sets and the accumulators exceed the
  // register file -- the 8-wave 256 x 256 tile with the dgrad epilogue's 16-float sets (128 + 128 VGPRs)
  // spilled 60 VGPRs to scratch; there the next block's operands are fetched after this block's emits.
  constexpr int kAccRegs = TN * TM * 4, kPreRegs = 2 * QR * (int)(sizeof(Pre) / 4);
  constexpr int PD = (HasFetch<EPI>::value && kAccRegs + kPreRegs > 224 && !TMAE_EPI_DEEP_ALWAYS) ? 1 : 2;
  Pre pf[PD][QR];
#pragma unroll
  for (int q = 0; q < QR; ++q) epi_fetch(e, m0 + q * RPI + rr, ncol, M, N, pf[0][q]);
#pragma unroll
  for (int j = 0; j < TM; ++j) {
#pragma unroll
    for (int i = 0; i < TN; ++i) *reinterpret_cast<f32x4*>(region + fr * ST + 16 * i + 4 * fq) = acc[i][j];
    if (PD == 2 && j + 1 < TM) {
#pragma unroll
      for (int q = 0; q < QR; ++q) epi_fetch(e, m0 + 16 * (j + 1) + q * RPI + rr, ncol, M, N, pf[(j + 1) % PD][q]);
    }
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int row = q * RPI + rr;
      const float* src = region + row * ST + 8 * cc;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
      const int m = m0 + 16 * j + row;
      if (m < M) epi_emit8_pre(e, m, ncol, lo, hi, N, pf[j % PD][q]);
    }
    if (PD == 1 && j + 1 < TM) {
#pragma unroll
      for (int q = 0; q < QR; ++q) epi_fetch(e, m0 + 16 * (j + 1) + q * RPI + rr, ncol, M, N, pf[0][q]);
    }
  }
}

// Plain bf16 stores (EpiStore<bf16, ACT> with no addend / pre-activation / f32 copy; N, ldo multiples of 8): bias and
// the activation are applied in the MFMA layout (each lane's 4 consecutive columns), the values rounded to bf16 and
// only THEN transposed through the wave's LDS region -- 8-B writes and half the read-back bytes of the f32 transpose
// (ds_write_b64 rows WN + 4 bf16 apart: conflict-free; ds_read_b128 2-way at most).  Same arithmetic per element as
// epilogue_lds + EpiStore::wide (acc + bias, the packed GELU, round to bf16): bitwise the same output.
template <class E, class = void> struct HasDirectBf16 : std::false_type {};
template <class E>
struct HasDirectBf16<E, std::enable_if_t<E::kDirectBf16>> : std::true_type {};

template <int TN, int TM, int WN, class EPI>
__device__ __forceinline__ void epilogue_lds_bf16(const EPI& e, const f32x4 (&acc)[TN][TM], bf16* region, int n0,
                                                  int m0, int lane, int M, int N) {
  constexpr int ST = WN + 4;     // row stride (bf16)
  constexpr int LPR = WN / 8;    // lanes per row (8 bf16 = 16 B each)
  constexpr int RPI = 64 / LPR;  // rows per read round
  constexpr int QR = 16 / RPI;   // read rounds per 16-row block
  const int fr = lane & 15, fq = lane >> 4;
  const int rr = lane / LPR, cc = lane - rr * LPR;
  f32x4 bv[TN];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + 16 * i + 4 * fq;
    bv[i] = (e.bias && n < N) ? load4f(e.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int ncol = n0 + 8 * cc;
#pragma unroll
  for (int j = 0; j < TM; ++j) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      f32x4 v = acc[i][j] + bv[i];
      if constexpr (EPI::kAct == TMAE_ACT_GELU) {
        v.xy = gelu2_bf16out(v.xy);
        v.zw = gelu2_bf16out(v.zw);
      }
      if constexpr (EPI::kAct == TMAE_ACT_RELU) {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.0f);
      }
      bf16x4 q;
      q[0] = (bf16)v[0]; q[1] = (bf16)v[1]; q[2] = (bf16)v[2]; q[3] = (bf16)v[3];
      *reinterpret_cast<bf16x4*>(region + fr * ST + 16 * i + 4 * fq) = q;
    }
#pragma unroll
    for (int q = 0; q < QR; ++q) {
      const int row = q * RPI + rr;
      const uint4 val = *reinterpret_cast<const uint4*>(region + row * ST + 8 * cc);
      const int m = m0 + 16 * j + row;
      if (m < M && ncol < N) *reinterpret_cast<uint4*>(e.out + (size_t)m * e.ldo + ncol) = val;
    }
  }
}

// the epilogue of one wave's tile: the bf16-first transpose when the functor allows it, else epilogue_lds
template <int TN, int TM, int WN, class EPI>
__device__ __forceinline__ void epilogue_any(const EPI& epi, const f32x4 (&acc)[TN][TM], float* region, int n0, int m0,
                                             int lane, int M, int N) {
  if constexpr (HasDirectBf16<EPI>::value && TMAE_EPI_BF16_DIRECT) {
    if (epi.direct_ok(N)) {  // wave-uniform
      epilogue_lds_bf16<TN, TM, WN>(epi, acc, reinterpret_cast<bf16*>(region), n0, m0, lane, M, N);
      return;
    }
  }
  epilogue_lds<TN, TM, WN>(epi, acc, region, n0, m0, lane, M, N);
}

// ------------------------------------------------------------------ timeline builds (tools/gemm_trace.py)
// -DTMAE_GEMM_TRACE=1: wave 0 of every workgroup of gemm_glds_kernel stamps the shader clock (s_memtime) at its
// start, after the prologue's DMA wait, after the K loop and after the epilogue, with its HW_ID / XCC_ID, into one
// row per workgroup of g_gemm_trace (read by tmae_gemm_trace_read in gemm.hip).
#ifndef TMAE_GEMM_TRACE
#define TMAE_GEMM_TRACE 0
#endif
#if TMAE_GEMM_TRACE
constexpr int GEMM_TR_WG = 8192, GEMM_TR_SLOTS = 8;
static __device__ unsigned long long g_gemm_trace[GEMM_TR_WG * GEMM_TR_SLOTS];
__device__ __forceinline__ void gemm_tr(int slot, unsigned long long v) {
  const int wg = blockIdx.x + gridDim.x * blockIdx.y;
  if (threadIdx.x == 0 && wg < GEMM_TR_WG) g_gemm_trace[(size_t)wg * GEMM_TR_SLOTS + slot] = v;
}
#define GEMM_TR(slot) gemm_tr(slot, __builtin_amdgcn_s_memtime())
#else
#define GEMM_TR(slot) ((void)0)
#endif

// ------------------------------------------------------------------ glds kernel
// One output tile per workgroup (XCD-aware tile order), 2-stage LDS ring: the next K-step's
// LDS-DMA is in flight under the current K-step's MFMAs.  After the last K-step the ring is reused
// as the epilogue's transpose buffer.  (A persistent walk with the next tile's first K-step in flight
// under the epilogue measured no better on the hot shapes and was dropped.)
// Also measured and dropped: a half-step software pipeline (second-half fragments loaded under the
// first half's MFMAs, the next step's first half under the second's, DMA two steps ahead): 1-3 %
// faster on isolated 8-wave GEMMs, 4 % slower on the whole forward (256 VGPRs on the 256 x 256 tile;
// the 4-wave tiles lost 5-8 % in isolation).
// counted DMA wait + raw barrier of the NS-stage ring: `younger` stages were issued after the one the next
// step reads (a __syncthreads fence would drain them too)
template <int PER, int NS>
__device__ __forceinline__ void gemm_ring_wait(int younger) {
  if (NS > 3 && younger >= 2)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * PER) : "memory");
  else if (younger >= 1)
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(PER) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// NS = LDS stages.  2: the next K-step's DMA in flight under the current MFMAs.  3 / 4 (small tiles, long K,
// e.g. the 6x6 / 3x3-grid LIC convs: a 32x64 tile's K-step is a few MFMAs, so a 2-stage ring pays the
// whole DMA latency every step): NS - 1 steps in flight.
template <typename T, int BN, int BM, int WGN, int NW, class WS, class XS, class EPI, int NS = 2>
__global__ void __launch_bounds__(64 * NW, NW == 8 ? 1 : 2)
gemm_glds_kernel(WS ws, XS xs, EPI epi, int M, int N, int K, int n2) {
  constexpr int BKE = 8 * Elt<T>::EPC;
  constexpr int WGM = NW / WGN;
  constexpr int WN = BN / WGN, WM = BM / WGM;
  constexpr int TN = WN / 16, TM = WM / 16;
  constexpr int PR = 8 * NW;                 // rows covered by one glds round of all waves
  // glds instructions per wave per stage; a token-side row count that is not a whole number of rounds (the
  // 8-wave 256 x 160 tile: 2.5 rounds of 64 rows) ends in a partial round issued by the first waves only
  constexpr int WJ = BN / PR, XJ = (BM + PR - 1) / PR;
  constexpr bool XPART = BM % PR != 0;
  constexpr int ROWS = BN + BM;
  static_assert(TN >= 1 && TM >= 1 && WJ >= 1 && XJ >= 1 && BN % PR == 0 && BM % 8 == 0, "bad tile");
  static_assert(!XPART || NS == 2, "partial DMA rounds need the uncounted 2-stage ring");
  static_assert(NS >= 2 && NS <= 4, "stages");
  __shared__ __attribute__((aligned(16))) uint4 lds[NS * ROWS * 8];

  GEMM_TR(0);
#if TMAE_GEMM_TRACE
  gemm_tr(4, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4));   // HW_ID
  gemm_tr(5, (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20));  // XCC_ID
#endif
  const int b1 = blockIdx.y / n2, b2 = blockIdx.y - (blockIdx.y / n2) * n2;
  ws.batch(b1, b2);
  xs.batch(b1, b2);
  epi.batch(b1, b2);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int nk = (K + BKE - 1) / BKE;

  const int lr = 8 * wave + (lane >> 3);
  const int pch = lane & 7;
  int wc[WJ], xc[XJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) wc[j] = pch ^ (((PR * j + lr) >> 1) & 7);
#pragma unroll
  for (int j = 0; j < XJ; ++j) xc[j] = pch ^ (((PR * j + lr) >> 1) & 7);
  typename WS::Row wrow[WJ];
  typename XS::Row xrow[XJ];
  // token-side K iterators (sources with one, the implicit conv): issue() below runs once per K-step, in order
  constexpr bool XIT = HasIter<XS>::value;
  struct NoIt {};
  using XIt = typename std::conditional<XIT, typename ItOf<XS, XIT>::type, NoIt>::type;
  XIt xit[XJ];
  auto set_rows = [&](int tn, int tm) {
#pragma unroll
    for (int j = 0; j < WJ; ++j) wrow[j] = ws.row(tn * BN + PR * j + lr);
#pragma unroll
    for (int j = 0; j < XJ; ++j) xrow[j] = xs.row(tm * BM + PR * j + lr);
    if constexpr (XIT)
#pragma unroll
      for (int j = 0; j < XJ; ++j) xit[j] = xs.iter(xrow[j], xc[j]);
  };
  const unsigned wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)lds;
  auto issue = [&](int stage, int kt) {
    const unsigned sb = lds_base + (unsigned)stage * ROWS * 128u;
    if constexpr (XIT) {
      if (kt * BKE + BKE <= K) {
#pragma unroll
        for (int j = 0; j < WJ; ++j)
          glds16(src_addr_full(ws, wrow[j], kt, wc[j]), sb + (unsigned)(PR * j + 8 * wave_u) * 128u);
      } else {
#pragma unroll
        for (int j = 0; j < WJ; ++j) glds16(ws.addr(wrow[j], kt, wc[j]), sb + (unsigned)(PR * j + 8 * wave_u) * 128u);
      }
#pragma unroll
      for (int j = 0; j < XJ; ++j) {
        const void* a = xs.next(xit[j]);  // every lane advances, including those of a partial round
        if (!XPART || PR * j + 8 * (int)wave_u < BM) glds16(a, sb + (unsigned)(BN + PR * j + 8 * wave_u) * 128u);
      }
      return;
    }
    if (kt * BKE + BKE <= K) {  // whole K-step: sources with addr_full skip the per-lane bounds select
#pragma unroll
      for (int j = 0; j < WJ; ++j)
        glds16(src_addr_full(ws, wrow[j], kt, wc[j]), sb + (unsigned)(PR * j + 8 * wave_u) * 128u);
#pragma unroll
      for (int j = 0; j < XJ; ++j)
        if (!XPART || PR * j + 8 * (int)wave_u < BM)
          glds16(src_addr_full(xs, xrow[j], kt, xc[j]), sb + (unsigned)(BN + PR * j + 8 * wave_u) * 128u);
    } else {
#pragma unroll
      for (int j = 0; j < WJ; ++j) glds16(ws.addr(wrow[j], kt, wc[j]), sb + (unsigned)(PR * j + 8 * wave_u) * 128u);
#pragma unroll
      for (int j = 0; j < XJ; ++j)
        if (!XPART || PR * j + 8 * (int)wave_u < BM)
          glds16(xs.addr(xrow[j], kt, xc[j]), sb + (unsigned)(BN + PR * j + 8 * wave_u) * 128u);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int tn, tm;
  tile_order(xcd_remap(blockIdx.x, gridDim.x), ntn, ntm, tn, tm);
  if (nk > 0 && NS == 2) {
    set_rows(tn, tm);
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    GEMM_TR(1);
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) issue(stage ^ 1, kt + 1);
      mfma_tile<T, BN, WN, WM, TN, TM>(lds + stage * ROWS * 8, wn, wm, lane, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stage ^= 1;
    }
  } else if (nk > 0) {
    // step kt reads stage kt % NS and issues step kt + NS - 1 into the stage step kt - 1 read (retired by
    // the barrier that closed step kt - 1)
    constexpr int PER = WJ + XJ;  // LDS-DMA instructions per wave per stage
    set_rows(tn, tm);
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nk) issue(s, s);
    gemm_ring_wait<PER, NS>(min(NS - 2, nk - 1));
    GEMM_TR(1);
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + NS - 1 < nk) issue((kt + NS - 1) % NS, kt + NS - 1);
      mfma_tile<T, BN, WN, WM, TN, TM>(lds + (kt % NS) * ROWS * 8, wn, wm, lane, acc);
      gemm_ring_wait<PER, NS>(min(kt + NS - 1, nk - 1) - (kt + 1));
    }
  }
  GEMM_TR(2);
  static_assert(NW * EpiRegion<WN>::FLOATS * 4 <= NS * ROWS * 128, "epilogue region exceeds the LDS ring");
#if defined(TMAE_GEMM_DIAG) && (TMAE_GEMM_DIAG & 1)  // phase isolation builds: no epilogue (accumulators kept live)
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) asm volatile("" ::"v"(acc[i][j]));
  return;
#endif
  epilogue_any<TN, TM, WN>(epi, acc, reinterpret_cast<float*>(lds) + wave * EpiRegion<WN>::FLOATS,
                           tn * BN + wn * WN, tm * BM + wm * WM, lane, M, N);
  GEMM_TR(3);
#if TMAE_GEMM_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  GEMM_TR(6);  // wave 0's stores complete
#endif
}

// ------------------------------------------------------------------ register-staged kernel
template <typename T, int BN, int BM, int WGN, class WS, class XS, class EPI>
__global__ void __launch_bounds__(256, 2)
gemm_reg_kernel(WS ws, XS xs, EPI epi, int M, int N, int K, int n2) {
  constexpr int BKE = 8 * Elt<T>::EPC;
  constexpr int WGM = 4 / WGN;
  constexpr int WN = BN / WGN, WM = BM / WGM;
  constexpr int TN = WN / 16, TM = WM / 16;
  constexpr int WCH = BN / 32, XCH = BM / 32;
  constexpr int ROWS = BN + BM;
  __shared__ __attribute__((aligned(16))) uint4 lds[2 * ROWS * 8];

  const int b1 = blockIdx.y / n2, b2 = blockIdx.y - (blockIdx.y / n2) * n2;
  ws.batch(b1, b2);
  xs.batch(b1, b2);
  epi.batch(b1, b2);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  int tn, tm;
  tile_order(xcd_remap(blockIdx.x, gridDim.x), (N + BN - 1) / BN, (M + BM - 1) / BM, tn, tm);
  const int n0 = tn * BN, m0 = tm * BM;
  const int ch = tid & 7, r0 = tid >> 3;

  typename WS::Row wrow[WCH];
  typename XS::Row xrow[XCH];
#pragma unroll
  for (int p = 0; p < WCH; ++p) wrow[p] = ws.row(n0 + r0 + 32 * p);
#pragma unroll
  for (int p = 0; p < XCH; ++p) xrow[p] = xs.row(m0 + r0 + 32 * p);
  uint4 wreg[WCH], xreg[XCH];
  auto gload = [&](int kt) {
#pragma unroll
    for (int p = 0; p < WCH; ++p) wreg[p] = ws.load(wrow[p], kt, ch);
#pragma unroll
    for (int p = 0; p < XCH; ++p) xreg[p] = xs.load(xrow[p], kt, ch);
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
  const int nk = (K + BKE - 1) / BKE;
  if (nk > 0) {
    gload(0);
    swrite(0);
  }
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) gload(kt + 1);
    mfma_tile<T, BN, WN, WM, TN, TM>(lds + (kt & 1) * ROWS * 8, wn, wm, lane, acc);
    if (kt + 1 < nk) swrite((kt + 1) & 1);
    __syncthreads();
  }
  static_assert(4 * EpiRegion<WN>::FLOATS * 4 <= 2 * ROWS * 128, "epilogue region exceeds the LDS ring");
  epilogue_any<TN, TM, WN>(epi, acc, reinterpret_cast<float*>(lds) + wave * EpiRegion<WN>::FLOATS, n0 + wn * WN,
                           m0 + wm * WM, lane, M, N);
}

// ------------------------------------------------------------------ launch with tile selection
struct TileChoice { int bn, bm, nw; };

// Tile candidates: 4-wave tiles run 2 workgroups per CU, the 8-wave 256x256 / 256x192 tiles one (128 KiB LDS).
// Score = (useful fraction of the padded MFMA work) x (tail quantisation: tiles / (rounds x slots))
// x (relative per-CU throughput of the tile shape at full occupancy).
// The 8-wave 256 x 192 tile (waves 2 x 4, 128 x 48 each) exists for the tail: 9280- and 16448-row token
// GEMMs whose 256 x 256 tile count lands just past a multiple of 256 CUs (enc qkv 333 tiles = 1.3
// rounds, dec fc1 520 = 2.03, dec proj/fc2 130 = 0.5).
static constexpr int kNumTiles = 9;
static constexpr int kTileCand[kNumTiles][3] = {{256, 256, 8}, {128, 128, 4}, {64, 128, 4}, {32, 128, 4}, {64, 64, 4},
                                                {32, 64, 4},   {256, 192, 8}, {128, 160, 4}, {128, 192, 4}};
// candidates only the bf16 LDS-DMA path instantiates
static inline bool tile_bf16_only(int i) { return kTileCand[i][2] == 8 || i >= 7; }
// eff = per-CU throughput relative to two 128 x 128 workgroups.  Forced-tile runs of the bench's token
// GEMMs (tools/gemm_bench.py) put the 8-wave tiles at 0.94-1.09 of it per CU at K <= 768 (two 4-wave
// workgroups per CU overlap one's epilogue with the other's main loop) and 1.24x at K = 3072 (fragment
// reuse amortising prologue / epilogue): eff(K) = e * (1 + 0.12 log2(K / 768)), with e (1.10 for
// 256x256, 1.08 for 256x192) picked by whole-forward A/B runs (bench.py: 8.57 ms vs 8.63 at 0.97 /
// 0.96 and 8.83 at 1.45 / 1.38).  The tile count's tail (ceil of rounds) decides the rest.
// The 4-wave 128 x 160 tile (waves 2 x 2, 64 x 80 each; 72 KiB LDS, two per CU) fits the token counts:
// 9280 = 58 x 160 and 16448 = 102.8 x 160 rows, where 128-row tiles leave a 2-4 % tail or a few
// workgroups past a full round (dec proj/fc2: 516 tiles for 512 slots).  Forced-tile runs: best on
// dec qkv / fc1 / fc2 / proj and enc fc1 (dec fc2 39.7 us vs 49.4 on 256 x 192); e160 = 1.22 from the
// constraints those runs put on the score and a whole-forward A/B (8070 img/s vs 8060 at 1.10, 7940 at
// 1.35, 7824 without the tile).
// 128 x 192 (waves 2 x 2, 64 x 96 each; 80 KiB LDS, exactly two per CU): enc qkv 42.2 us vs 49.6 on
// 256 x 192, dec fc1 54.6 vs 56.4 on 128 x 160; e = 1.25 inside the (1.10, 1.46) window those runs
// leave (whole forward 8108 img/s vs 8041 without it).  Round 3 re-check at HEAD (profiles/r03/
// s2_gemm_tiles_c13.log, s2_knob_c13_*): the pick within 3 % of the best forced tile on every token GEMM;
// the efficiencies moved by +-20 % changed the forward by -2 % .. +0.3 %.  (192 x 128 never won: dropped.)
// Round 4: an 8-wave 256 x 160 tile (half the L2 -> LDS bytes per MFMA of 2 x 128 x 160) measured slower when
// forced (enc fc1 65.0 vs 63.5 us, dec fc1 66.2 vs 57.3) and -6.5 % on the forward when offered to the chooser
// (profiles/r04/c9_*): dropped; the partial token-side DMA round it needed stays in the kernel.
// Tuning experiments override these with a variant build (tools/build_variant.sh -DTMAE_GEMM_TILE=<i>).
#ifndef TMAE_GEMM_TILE
#define TMAE_GEMM_TILE -1
#endif
static inline TileChoice choose_tile(int M, int N, int K, int batch, bool allow_big) {
  const double kf = 1.0 + 0.12 * std::log2(std::max(K, 768) / 768.0);
  const double eff[kNumTiles] = {1.10 * kf, 1.0, 0.86, 0.70, 0.72, 0.55, 1.08 * kf, 1.22, 1.25};
  constexpr int forced = TMAE_GEMM_TILE;
  if (forced >= 0 && forced < kNumTiles && (allow_big || !tile_bf16_only(forced)))
    return TileChoice{kTileCand[forced][0], kTileCand[forced][1], kTileCand[forced][2]};
  double best = -1.0;
  TileChoice tc{128, 128, 4};
  for (int i = 0; i < kNumTiles; ++i) {
    if (tile_bf16_only(i) && !allow_big) continue;
    const int bn = kTileCand[i][0], bm = kTileCand[i][1];
    const double tn = ceil_div(N, bn), tm = ceil_div(M, bm);
    const double useful = ((double)N / (tn * bn)) * ((double)M / (tm * bm));
    const double wgs = tn * tm * batch;
    const double slots = kTileCand[i][2] == 8 ? 256.0 : 512.0;
    const double quant = wgs / (std::ceil(wgs / slots) * slots);
    const double score = useful * quant * eff[i];
    if (score > best + 1e-9) { best = score; tc = TileChoice{bn, bm, kTileCand[i][2]}; }
  }
  return tc;
}

template <bool GLDS, typename T, int BN, int BM, int WGN, int NW, class WS, class XS, class EPI>
static int launch_one(const char* name, const WS& ws, const XS& xs, const EPI& epi, int M, int N, int K, int n1,
                      int n2, hipStream_t st) {
  const int tiles = ceil_div(N, BN) * ceil_div(M, BM);
  if (tiles == 0 || n1 * n2 == 0) return TMAE_OK;
  if constexpr (GLDS) {
    // small tiles over a long K take a 4-stage (<= 160 LDS rows) or 3-stage (<= 213 rows) ring: either stays
    // within 80 KB, two workgroups per CU (LIC conv family 1129 -> 1095 us per forward)
    constexpr int DNS = (BN + BM) * 128 * 4 <= 80 * 1024 ? 4 : (BN + BM) * 128 * 3 <= 80 * 1024 ? 3 : 2;
    constexpr bool deep_ok = sizeof(T) == 2 && NW == 4 && DNS > 2;
    if constexpr (deep_ok) {
      if (ceil_div(K, 8 * Elt<T>::EPC) >= 8) {
        hipLaunchKernelGGL((gemm_glds_kernel<T, BN, BM, WGN, NW, WS, XS, EPI, DNS>), dim3(tiles, n1 * n2),
                           dim3(64 * NW), 0, st, ws, xs, epi, M, N, K, n2);
        TMAE_LAUNCH_CHECK(name);
      }
    }
    hipLaunchKernelGGL((gemm_glds_kernel<T, BN, BM, WGN, NW, WS, XS, EPI>), dim3(tiles, n1 * n2), dim3(64 * NW), 0,
                       st, ws, xs, epi, M, N, K, n2);
  } else {
    hipLaunchKernelGGL((gemm_reg_kernel<T, BN, BM, WGN, WS, XS, EPI>), dim3(tiles, n1 * n2), dim3(256), 0, st, ws, xs,
                       epi, M, N, K, n2);
  }
  TMAE_LAUNCH_CHECK(name);
}

template <bool GLDS, typename T, class XS, class EPI>
static int launch_gemm(const char* name, const T* w, long long ws1, long long ws2, int N, int K, const XS& xs,
                       const EPI& epi, int M, int n1 = 1, int n2 = 1, hipStream_t st = 0) {
  DenseSrc<T> ws{w, K, N, K, 1 << 30, 0, 0, BStride{ws1, ws2}};
  // the 8-wave tile is built for the bf16 glds path only (the f32 path is the parity path)
  const TileChoice tc = choose_tile(M, N, K, n1 * n2, GLDS && sizeof(T) == 2);
  if constexpr (GLDS && sizeof(T) == 2) {
    if (tc.nw == 8 && tc.bm == 192) return launch_one<GLDS, T, 256, 192, 2, 8>(name, ws, xs, epi, M, N, K, n1, n2, st);
    if (tc.nw == 4 && tc.bm == 160) return launch_one<GLDS, T, 128, 160, 2, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
    if (tc.nw == 4 && tc.bm == 192) return launch_one<GLDS, T, 128, 192, 2, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
    if (tc.nw == 8) return launch_one<GLDS, T, 256, 256, 2, 8>(name, ws, xs, epi, M, N, K, n1, n2, st);
  }
  if (tc.bn == 128) return launch_one<GLDS, T, 128, 128, 2, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
  if (tc.bn == 64 && tc.bm == 128) return launch_one<GLDS, T, 64, 128, 1, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
  if (tc.bn == 32 && tc.bm == 128) return launch_one<GLDS, T, 32, 128, 1, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
  if (tc.bn == 64) return launch_one<GLDS, T, 64, 64, 2, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
  return launch_one<GLDS, T, 32, 64, 1, 4>(name, ws, xs, epi, M, N, K, n1, n2, st);
}

// ------------------------------------------------------------------ shared epilogues
// out[m][n..n+3] = act(acc + bias (+ addend[m][n])) in OT; optional second f32 copy (out32).
template <typename OT, int ACT> struct EpiStore {
  static constexpr bool kDirectBf16 = sizeof(OT) == 2;  // epilogue_lds_bf16 (when direct_ok)
  static constexpr int kAct = ACT;
  OT* out;
  int ldo;
  const float* bias;
  const float* addend;  // optional pre-activation addend (precomputed partial sums)
  int ld_add;
  float* out32;         // optional f32 copy
  int ld32;
  OT* pre;              // optional pre-activation copy (training keeps GELU inputs for the backward)
  int ldp;
  BStride so, sb, sa, s32, sp;
  __device__ void batch(int b1, int b2) {
    out += so.at(b1, b2);
    if (bias) bias += sb.at(b1, b2);
    if (addend) addend += sa.at(b1, b2);
    if (out32) out32 += s32.at(b1, b2);
    if (pre) pre += sp.at(b1, b2);
  }
  __device__ void operator()(int m, int n, f32x4 v) const {
    if (bias) v += load4f(bias + n);
    if (addend) v += load4f(addend + (size_t)m * ld_add + n);
    if (pre) store4(pre + (size_t)m * ldp + n, v);
    if (ACT == TMAE_ACT_GELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = gelu_for<OT>(v[j]);
    }
    if (ACT == TMAE_ACT_RELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j], 0.0f);
    }
    store4(out + (size_t)m * ldo + n, v);
    if (out32) store4(out32 + (size_t)m * ld32 + n, v);
  }
  __device__ bool direct_ok(int N) const {
    return !addend && !pre && !out32 && (N & 7) == 0 && (ldo & 7) == 0 && ((uintptr_t)out & 15) == 0;
  }
  // epilogue_lds hooks: this lane's bias columns once, the addend one row block ahead
  f32x4 pb0, pb1;
  __device__ void prefetch(int n, int N) {
    pb0 = pb1 = f32x4{0.f, 0.f, 0.f, 0.f};
    if (bias && n + 8 <= N) load8f(bias + n, pb0, pb1);
  }
  struct Pre { f32x4 a0, a1; };
  __device__ Pre fetch(int m, int n) const {
    Pre p;
    if (addend) load8f(addend + (size_t)m * ld_add + n, p.a0, p.a1);
    return p;
  }
  __device__ void wide(int m, int n, f32x4 lo, f32x4 hi, const Pre& p) const {
    lo += pb0; hi += pb1;
    if (addend) { lo += p.a0; hi += p.a1; }
    if (pre) store8(pre + (size_t)m * ldp + n, lo, hi);
    if (ACT == TMAE_ACT_GELU) {
      if constexpr (sizeof(OT) == 2) {
        gelu8_bf16out(lo, hi);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { lo[j] = gelu_for<OT>(lo[j]); hi[j] = gelu_for<OT>(hi[j]); }
      }
    }
    if (ACT == TMAE_ACT_RELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { lo[j] = fmaxf(lo[j], 0.0f); hi[j] = fmaxf(hi[j], 0.0f); }
    }
    store8(out + (size_t)m * ldo + n, lo, hi);
    if (out32) store8(out32 + (size_t)m * ld32 + n, lo, hi);
  }};

template <typename OT, int ACT>
static inline EpiStore<OT, ACT> make_store(OT* out, int ldo, const float* bias) {
  EpiStore<OT, ACT> e;
  e.out = out; e.ldo = ldo; e.bias = bias; e.addend = nullptr; e.ld_add = 0; e.out32 = nullptr; e.ld32 = 0;
  e.pre = nullptr; e.ldp = 0;
  e.so = e.sb = e.sa = e.s32 = e.sp = BStride{0, 0};
  return e;
}
