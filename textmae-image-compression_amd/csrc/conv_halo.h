// 3x3 stride-1 convolution over 12x12 NHWC maps with the input halo staged in LDS (bf16).
//
// Every LIC conv of the slice loop (cc_transform_mean/scale, lrp_transform; MCM.py:165-293, 761-784),
// h_a's first two layers and h_s's last layer (MCM.py:115-162) runs on the 12x12 latent grid.  The
// implicit-GEMM path (gemm_glds_kernel + ConvSrc) re-fetches every input row once per tap, i.e. nine
// times per K sweep, through L2, with tiles small enough (N <= 224 output channels) that address math
// and LDS-DMA issue dominate its K-steps.  Here one workgroup owns ONE image x BN output channels:
//   per 64-channel input chunk: the zero-padded 14x14 halo of that image goes global -> LDS once
//                               (LDS-DMA, 16-B pieces, row-swizzled like the GEMM core);
//   per (chunk, tap) K-step:    the BN x 64 weight slab of that tap streams into a 2-stage LDS ring and
//                               the 144 output pixels read their shifted halo rows straight from LDS.
// MFMA v_mfma_f32_16x16x32_bf16 issued swapped (A = weight rows, B = pixel rows) exactly as the GEMM
// core, so the accumulator layout, the LDS-transposed epilogue (epilogue_lds) and every epilogue
// functor (bias / GELU / addend / f32 copy / LRP) are shared with it.  4 waves: 2 along N x 2 along M,
// each wave 5 M-fragments (160 rows >= 144; rows >= 144 are computed on a clamped halo row and dropped).
#pragma once

#include "gemm_core.h"

namespace halo {
constexpr int G = 12;          // map side
constexpr int HP = 14;         // halo side
constexpr int PIX = G * G;     // 144 output rows per image
constexpr int HROWS = 224;     // halo rows staged (196 used), 28 LDS-DMA rounds of 8 rows
constexpr int TMF = 5;         // M fragments per wave
}  // namespace halo

// channels [0, c1) of a pixel from x1 (row stride ld1), [c1, Cin) from x2 (torch.cat without a copy)
struct HaloSrc {
  const bf16* x1;
  const bf16* x2;
  int c1, ld1, ld2, Cin;
  BStride bs1, bs2;
  __device__ void batch(int b1, int b2) {
    x1 += bs1.at(b1, b2);
    x2 += bs2.at(b1, b2);
  }
  // halo row hr (= hy * 14 + hx) of image img, 8 channels from ch; zero outside the map / channel range
  __device__ const void* addr(int img, int hr, int ch) const {
    if (hr >= halo::HP * halo::HP || ch >= Cin) return g_tmae_zero_page;
    const int hy = hr / halo::HP;
    const int iy = hy - 1, ix = hr - hy * halo::HP - 1;
    if ((unsigned)iy >= (unsigned)halo::G || (unsigned)ix >= (unsigned)halo::G) return g_tmae_zero_page;
    const size_t pix = (size_t)img * halo::PIX + iy * halo::G + ix;
    return ch < c1 ? (const void*)(x1 + pix * ld1 + ch) : (const void*)(x2 + pix * ld2 + (ch - c1));
  }
};

// counted wait: every LDS-DMA but the wave's N youngest has landed, then the workgroup barrier (a
// __syncthreads fence would drain the look-ahead DMA too)
template <int N>
__device__ __forceinline__ void halo_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Pipeline: weights in a 3-slot ring (the slab of step k+2 is issued while step k computes, so each DMA
// has a whole K-step of slack), halo in 2 slots (chunk c+1 issued at tap 0 of chunk c).  LDS: BN=64
// 3 x 8 KiB + 2 x 28 KiB = 80 KiB (two workgroups per CU), BN=128 104 KiB (one).
template <int BN, class EPI>
__global__ void __launch_bounds__(256, BN == 64 ? 2 : 1)
conv_halo_kernel(const bf16* __restrict__ w, BStride wst, HaloSrc src, EPI epi, int N, int n2) {
  using namespace halo;
  constexpr int WN = BN / 2, TN = WN / 16;
  constexpr int NWS = 3;  // weight ring slots
  constexpr int WBYTES = BN * 128, HBYTES = HROWS * 128, HOFF = NWS * WBYTES;
  constexpr int WJ = BN / 32, HJ = HROWS / 32;  // LDS-DMA rounds per wave (4 waves x 8 rows each)
  static_assert(TN >= 2 && WN % 32 == 0, "conv_halo: tile");
  static_assert(4 * EpiRegion<WN>::FLOATS * 4 <= NWS * WBYTES + 2 * HBYTES, "conv_halo: epilogue region");
  __shared__ __attribute__((aligned(16))) uint4 lds[(NWS * WBYTES + 2 * HBYTES) / 16];

  const int b1 = blockIdx.y / n2, b2 = blockIdx.y - (blockIdx.y / n2) * n2;
  w += wst.at(b1, b2);
  src.batch(b1, b2);
  epi.batch(b1, b2);
  const int Cin = src.Cin, ldw = 9 * Cin;
  const int ntn = (N + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int img = t / ntn, tn = t - img * ntn;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int nchunk = (Cin + 63) >> 6, nk = 9 * nchunk;

  // LDS-DMA roles: one glds16 moves 8 LDS rows x 128 B; lane -> row +(lane >> 3), 16-B slot (lane & 7).
  // Slot s of row r holds source chunk s ^ ((r >> 1) & 7) (the GEMM core's swizzle).
  const int lr = lane >> 3, pch = lane & 7;
  const unsigned wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)lds;
  const bf16* wrow[WJ];
  int wch[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) {
    const int r = 8 * (wave + 4 * j) + lr, n = tn * BN + r;
    wrow[j] = n < N ? w + (size_t)n * ldw : nullptr;
    wch[j] = 8 * (pch ^ ((r >> 1) & 7));
  }
  auto issue_w = [&](int stage, int kk) {
    const int chunk = kk / 9, tap = kk - 9 * chunk;
    const unsigned sb = lds_base + (unsigned)stage * WBYTES;
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      const int ch = 64 * chunk + wch[j];
      const void* s = (wrow[j] && ch < Cin) ? (const void*)(wrow[j] + tap * Cin + ch) : (const void*)g_tmae_zero_page;
      glds16(s, sb + (8u * (wave_u + 4u * j)) * 128u);
    }
  };
  auto issue_h = [&](int stage, int chunk) {
    const unsigned sb = lds_base + (unsigned)HOFF + (unsigned)stage * HBYTES;
#pragma unroll
    for (int j = 0; j < HJ; ++j) {
      const int r = 8 * (wave + 4 * j) + lr;
      glds16(src.addr(img, r, 64 * chunk + 8 * (pch ^ ((r >> 1) & 7))), sb + (8u * (wave_u + 4u * j)) * 128u);
    }
  };

  f32x4 acc[TN][TMF];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TMF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  int hr0[TMF];  // halo row of tap (0, 0) for this lane's pixel in each M fragment
#pragma unroll
  for (int j = 0; j < TMF; ++j) {
    const int p = 16 * (wm * TMF + j) + fr;
    const int y = p / G;
    hr0[j] = p < PIX ? y * HP + (p - y * G) : 0;
  }

  if (nk > 0) {
    // prologue: halo(0), w(0) landed; w(1) may stay in flight
    issue_h(0, 0);
    issue_w(0, 0);
    if (nk > 1) {
      issue_w(1, 1);
      halo_wait_barrier<WJ>();
    } else {
      halo_wait_barrier<0>();
    }
    int chunk = 0, tap = 0, wslot = 0;
    for (int kk = 0; kk < nk; ++kk) {
      // slot (kk+2)%3 was last read by step kk-1, retired by the barrier that closed it
      const bool more = kk + 2 < nk;
      if (more) issue_w(wslot == 0 ? 2 : wslot - 1, kk + 2);
      const bool hnext = tap == 0 && chunk + 1 < nchunk;  // implies `more` (9 steps per chunk)
      if (hnext) issue_h((chunk + 1) & 1, chunk + 1);
      const uint4* wb = lds + wslot * (WBYTES / 16);
      const unsigned char* hb = reinterpret_cast<const unsigned char*>(lds) + HOFF + (chunk & 1) * HBYTES;
      const int ky = (tap * 11) >> 5;  // tap / 3
      const int toff = ky * HP + (tap - 3 * ky);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = 4 * s + fq;
        bf16x8 a[TN], b[TMF];
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int r = wn * WN + 16 * i + fr;
          uint4 u = wb[r * 8 + (c ^ ((r >> 1) & 7))];
          a[i] = *reinterpret_cast<bf16x8*>(&u);
        }
#pragma unroll
        for (int j = 0; j < TMF; ++j) {
          const int hr = hr0[j] + toff;
          uint4 u = *reinterpret_cast<const uint4*>(hb + hr * 128 + 16 * (c ^ ((hr >> 1) & 7)));
          b[j] = *reinterpret_cast<bf16x8*>(&u);
        }
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TMF; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
      // w(kk+1) must have landed for the next step; this step's own issues (w(kk+2), halo) stay in flight
      if (hnext) halo_wait_barrier<WJ + HJ>();
      else if (more) halo_wait_barrier<WJ>();
      else halo_wait_barrier<0>();
      wslot = wslot == NWS - 1 ? 0 : wslot + 1;
      if (++tap == 9) {
        tap = 0;
        ++chunk;
      }
    }
  }
  // rows >= 144 of the last fragments belong to no pixel: the epilogue's row limit drops them
  epilogue_lds<TN, TMF, WN>(epi, acc, reinterpret_cast<float*>(lds) + wave * EpiRegion<WN>::FLOATS, tn * BN + wn * WN,
                            img * PIX + wm * (16 * TMF), lane, (img + 1) * PIX, N);
}

// BN: the tile with the least channel padding; 64 when 128 would leave the chip short of workgroups
static inline int conv_halo_bn(int N, int nimg, int nb) {
  const int forced = gemm_knob("TMAE_CONV_HALO_BN", 0);
  if (forced == 64 || forced == 128) return forced;
  const int t128 = ceil_div(N, 128), t64 = ceil_div(N, 64);
  if (t64 * 64 < t128 * 128) return 64;
  if ((long long)nimg * t128 * nb < 256) return 64;
  return 128;
}

// eligible: bf16, stride 1, 12x12, at most TMAE_CONV_HALO_MAXN output channels (default 512: the wide
// latent-precompute convs stay on the 256x256 GEMM tile) and TMAE_CONV_HALO_MAXNB problems per launch
// (default 2: the 12-problem launches of slices 6..11 fill the chip with 256x256 GEMM tiles, measured
// faster); TMAE_CONV_HALO=0 disables
static inline bool conv_halo_ok(int H, int W, int stride, int N, int nb) {
  const int on = gemm_knob("TMAE_CONV_HALO", 1);
  const int maxn = gemm_knob("TMAE_CONV_HALO_MAXN", 512);
  const int maxnb = gemm_knob("TMAE_CONV_HALO_MAXNB", 2);
  return on && H == halo::G && W == halo::G && stride == 1 && N <= maxn && nb <= maxnb;
}

template <class EPI>
static int launch_conv_halo(const char* name, const bf16* w, BStride wst, const HaloSrc& src, const EPI& epi, int N,
                            int nimg, int nb1, int nb2, hipStream_t st) {
  if (N == 0 || nimg == 0 || nb1 * nb2 == 0) return TMAE_OK;
  const int bn = conv_halo_bn(N, nimg, nb1 * nb2);
  const dim3 grid(nimg * ceil_div(N, bn), nb1 * nb2);
  if (bn == 64)
    hipLaunchKernelGGL((conv_halo_kernel<64, EPI>), grid, dim3(256), 0, st, w, wst, src, epi, N, nb2);
  else
    hipLaunchKernelGGL((conv_halo_kernel<128, EPI>), grid, dim3(256), 0, st, w, wst, src, epi, N, nb2);
  TMAE_LAUNCH_CHECK(name);
}
