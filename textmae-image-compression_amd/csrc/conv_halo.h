// 3x3 stride-1 convolution over 12x12 NHWC maps with the input halo staged in LDS (bf16).
//
// Every LIC conv of the slice loop (cc_transform_mean/scale, lrp_transform; MCM.py:165-293, 761-784),
// h_a's first two layers and h_s's last layer (MCM.py:115-162) runs on the 12x12 latent grid.  The
// implicit-GEMM path (gemm_glds_kernel + ConvSrc) re-fetches every input row once per tap, i.e. nine
// times per K sweep, through L2, with tiles small enough (N <= 224 output channels) that address math
// and LDS-DMA issue dominate its K-steps.  Here one workgroup owns ONE image x BN output channels:
//   per 64-channel input chunk: the zero-padded 14x14 halo of that image goes global -> LDS once
//                               (LDS-DMA, 16-B pieces);
//   per (chunk, tap) K-step:    the BN x 64 weight slab of that tap streams into a 3-slot LDS ring and
//                               the 144 output pixels read their shifted halo rows straight from LDS.
// MFMA v_mfma_f32_16x16x32_bf16 issued swapped (A = weight rows, B = pixel rows) as in the GEMM core,
// so every epilogue functor (bias / GELU / addend / f32 copy / LRP) is shared with it.
//
// Addressing is built so the K loop carries no address arithmetic (PMC on the first version: 5 VALU
// and 4 SALU instructions per MFMA, 38 % of LDS cycles lost to bank conflicts):
//   * halo rows are LINEAR with a 144-B pitch (128 B of channels + 16 B pad), so the halo row of tap
//     (ky, kx) is the tap-(0,0) row + (14 ky + kx) rows: with the nine taps unrolled every fragment
//     read is a per-lane base + a compile-time offset (ds_read_b128 offset field);
//   * an MFMA M-fragment is a 4x4 pixel block (9 blocks tile the 12x12 map): with the 144-B pitch
//     its reads are 2-way bank conflicted at worst for every tap (tools: exhaustive check over the
//     gfx950 ds_read_b128 lane groups; no 16-B layout is conflict-free because a lane group mixes two
//     k-chunks), and the epilogue maps fragment rows back to pixels;
//   * the weight ring slot of tap t is t % 3 (nine taps per chunk), also compile-time.
// 4 waves: 2 along N x 2 along M, 5 M-fragments each (block 9 of the second M-wave is padding).
#pragma once

#include "gemm_core.h"

namespace halo {
constexpr int G = 12;                      // map side
constexpr int HP = 14;                     // halo side
constexpr int PIX = G * G;                 // 144 output pixels per image
constexpr int HR = HP * HP;                // 196 halo rows
constexpr int PITCH = 144;                 // bytes per halo row (8 channel chunks + 1 pad chunk)
constexpr int HCH = HR * (PITCH / 16);     // 16-B LDS chunks of one halo image (pads included)
constexpr int HJ = (HCH + 255) / 256;      // LDS-DMA rounds per wave (4 waves x 64 lanes) = 7
constexpr int HSLOT = HJ * 256 * 16;       // bytes of one halo slot (tail of the last round included)
constexpr int TMF = 5;                     // M fragments per wave
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
  // pixel pix (image-major) channels [ch, ch + 8); zero page for padding / out-of-range channels
  __device__ const void* addr(int pix, int ch) const {
    if (pix < 0 || ch >= Cin) return g_tmae_zero_page;
    return ch < c1 ? (const void*)(x1 + (size_t)pix * ld1 + ch) : (const void*)(x2 + (size_t)pix * ld2 + (ch - c1));
  }
};

// counted wait: every LDS-DMA but the wave's N youngest has landed, then the workgroup barrier (a
// __syncthreads fence would drain the look-ahead DMA too)
template <int N>
__device__ __forceinline__ void halo_wait_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// Epilogue through each wave's LDS region (as epilogue_lds in gemm_core.h): fragment f = 4x4 block
// (f / 3, f % 3); transposed row `row` of a fragment is pixel (4 by + row / 4, 4 bx + row % 4).
template <int TN, int WN, class EPI>
__device__ __forceinline__ void halo_epilogue(const EPI& epi, const f32x4 (&acc)[TN][halo::TMF], float* region, int n0,
                                              int img, int wm, int lane, int N) {
  constexpr int ST = EpiRegion<WN>::ST, LPR = WN / 8, RPI = 64 / LPR;
  const int fr = lane & 15, fq = lane >> 4;
  const int rr = lane / LPR, cc = lane - rr * LPR;
#pragma unroll
  for (int j = 0; j < halo::TMF; ++j) {
    const int f = wm * halo::TMF + j;
    if (f >= 9) break;  // wave-uniform
    const int by = f / 3, bx = f - 3 * by;
#pragma unroll
    for (int i = 0; i < TN; ++i) *reinterpret_cast<f32x4*>(region + fr * ST + 16 * i + 4 * fq) = acc[i][j];
#pragma unroll
    for (int q = 0; q < 16 / RPI; ++q) {
      const int row = q * RPI + rr;
      const float* src = region + row * ST + 8 * cc;
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
      const int p = (4 * by + (row >> 2)) * halo::G + 4 * bx + (row & 3);
      epi_emit8(epi, img * halo::PIX + p, n0 + 8 * cc, lo, hi, N);
    }
  }
}

// Pipeline: weights in a 3-slot ring (the slab of step k+2 is issued while step k computes: a whole
// K-step of slack per DMA), halo in 2 slots (chunk c+1 issued at tap 0 of chunk c).  LDS: BN=64
// 3 x 8 KiB + 2 x 28 KiB = 80 KiB (two workgroups per CU), BN=128 104 KiB (one).
template <int BN, class EPI>
__global__ void __launch_bounds__(256, BN == 64 ? 2 : 1)
conv_halo_kernel(const bf16* __restrict__ w, BStride wst, HaloSrc src, EPI epi, int N, int n2) {
  using namespace halo;
  constexpr int WN = BN / 2, TN = WN / 16;
  constexpr int NWS = 3;  // weight ring slots
  constexpr int WBYTES = BN * 128, HOFF = NWS * WBYTES;
  constexpr int WJ = BN / 32;  // weight LDS-DMA rounds per wave (4 waves x 8 rows each)
  static_assert(TN >= 2 && WN % 32 == 0, "conv_halo: tile");
  static_assert(4 * EpiRegion<WN>::FLOATS * 4 <= HOFF + 2 * HSLOT, "conv_halo: epilogue region");
  __shared__ __attribute__((aligned(16))) uint4 lds[(HOFF + 2 * HSLOT) / 16];
  const unsigned char* lb = reinterpret_cast<const unsigned char*>(lds);

  const int b1 = blockIdx.y / n2, b2 = blockIdx.y - (blockIdx.y / n2) * n2;
  w += wst.at(b1, b2);
  src.batch(b1, b2);
  epi.batch(b1, b2);
  const int Cin = src.Cin, ldw = 9 * Cin;
  const int ntn = (N + BN - 1) / BN;
  const int t0 = xcd_remap(blockIdx.x, gridDim.x);
  const int img = t0 / ntn, tn = t0 - img * ntn;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave & 1, wm = wave >> 1;
  const int nchunk = (Cin + 63) >> 6, nk = 9 * nchunk;
  const unsigned wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)lds;

  // weight DMA roles: glds16 = 8 LDS rows x 128 B; lane -> row +(lane >> 3), slot (lane & 7) holding
  // source chunk slot ^ ((row >> 1) & 7) (the GEMM core's swizzle)
  const int lr = lane >> 3, pch = lane & 7;
  const bf16* wrow[WJ];
  int wch[WJ];
#pragma unroll
  for (int j = 0; j < WJ; ++j) {
    const int r = 8 * (wave + 4 * j) + lr, n = tn * BN + r;
    wrow[j] = n < N ? w + (size_t)n * ldw : nullptr;
    wch[j] = 8 * (pch ^ ((r >> 1) & 7));
  }
  auto issue_w = [&](int slot, int chunk, int tap) {
    const unsigned sb = lds_base + (unsigned)slot * WBYTES;
#pragma unroll
    for (int j = 0; j < WJ; ++j) {
      const int ch = 64 * chunk + wch[j];
      const void* s = (wrow[j] && ch < Cin) ? (const void*)(wrow[j] + tap * Cin + ch) : (const void*)g_tmae_zero_page;
      glds16(s, sb + (8u * (wave_u + 4u * j)) * 128u);
    }
  };
  // halo DMA roles: 16-B chunk q = 64 (wave + 4 j) + lane of the linear image -> halo row q / 9,
  // channel chunk q % 9 (8 = the pad); source pixel (or -1 for the zero border / pads / tail)
  int hpix[HJ], hch[HJ];
#pragma unroll
  for (int j = 0; j < HJ; ++j) {
    const int q = 64 * (wave + 4 * j) + lane;
    const int row = q / 9, sl = q - 9 * row;
    const int hy = row / HP, hx = row - hy * HP;
    const bool ok = row < HR && sl < 8 && hy >= 1 && hy <= G && hx >= 1 && hx <= G;
    hpix[j] = ok ? img * PIX + (hy - 1) * G + (hx - 1) : -1;
    hch[j] = 8 * sl;
  }
  auto issue_h = [&](int slot, int chunk) {
    const unsigned sb = lds_base + (unsigned)HOFF + (unsigned)slot * HSLOT;
#pragma unroll
    for (int j = 0; j < HJ; ++j) glds16(src.addr(hpix[j], 64 * chunk + hch[j]), sb + 1024u * (wave_u + 4u * j));
  };

  // per-lane fragment read offsets (bytes): weights per (i, s), halo per j (tap (0,0), k-chunk fq)
  const int fr = lane & 15, fq = lane >> 4;
  int woff[TN][2];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r = wn * WN + 16 * i + fr;
      woff[i][s] = r * 128 + 16 * ((4 * s + fq) ^ ((r >> 1) & 7));
    }
  int hoff[TMF];
#pragma unroll
  for (int j = 0; j < TMF; ++j) {
    const int f = wm * TMF + j, by = f / 3, bx = f - 3 * by;
    const int y = 4 * by + (fr >> 2), x = 4 * bx + (fr & 3);
    hoff[j] = f < 9 ? (y * HP + x) * PITCH + 16 * fq : 16 * fq;  // padding block: any in-range rows
  }

  f32x4 acc[TN][TMF];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TMF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    // prologue: halo(0), w(0) landed; w(1) may stay in flight
    issue_h(0, 0);
    issue_w(0, 0, 0);
    issue_w(1, 0, 1);
    halo_wait_barrier<WJ>();
    for (int chunk = 0; chunk < nchunk; ++chunk) {
      const unsigned char* hb = lb + HOFF + (chunk & 1) * HSLOT;
      const bool last = chunk + 1 == nchunk;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        // slot (t+2)%3 was last read by the previous step, retired by the barrier that closed it
        const bool more = !last || t + 2 < 9;
        if (more) issue_w((t + 2) % 3, t + 2 < 9 ? chunk : chunk + 1, (t + 2) % 9);
        const bool hnext = t == 0 && !last;
        if (hnext) issue_h((chunk + 1) & 1, chunk + 1);
        const unsigned char* wb = lb + (t % 3) * WBYTES;
        const int toff = ((t / 3) * HP + (t % 3)) * PITCH;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          bf16x8 a[TN], b[TMF];
#pragma unroll
          for (int i = 0; i < TN; ++i) a[i] = *reinterpret_cast<const bf16x8*>(wb + woff[i][s]);
#pragma unroll
          for (int j = 0; j < TMF; ++j) b[j] = *reinterpret_cast<const bf16x8*>(hb + hoff[j] + toff + 64 * s);
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int j = 0; j < TMF; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        // w(next step) must have landed; this step's own issues (w(+2), halo) stay in flight
        if (hnext) halo_wait_barrier<WJ + HJ>();
        else if (more) halo_wait_barrier<WJ>();
        else halo_wait_barrier<0>();
      }
    }
  }
  halo_epilogue<TN, WN>(epi, acc, reinterpret_cast<float*>(lds) + wave * EpiRegion<WN>::FLOATS, tn * BN + wn * WN,
                        img, wm, lane, N);
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
