// Fused qkv projection + multi-head attention for the bf16 inference forward (timm Block attention branch,
// MCM.py:629-630 encoder, 678-679 decoder):   O = softmax(Q K^T * dh^-0.5) V,   [Q | K | V] = X W_qkv^T + b.
//
// Unfused, the qkv GEMM writes [B*T][3D] bf16 to HBM and the attention kernel reads it straight back
// (85 MB per encoder layer, 101 MB per decoder layer at batch 64), and the GEMM's store burst is the
// slowest part of its epilogue.  Here ONE workgroup owns (image b, head group g of HG heads):
//   1. GEMM: the tile is all Tpad (= T rounded up to 32) token rows of image b x the 3 * HG * dh weight rows
//      of its heads' q, k and v (192 columns for ViT-B dh 64 x 1 head and the decoder's dh 32 x 2 heads),
//      K = D; the same LDS-DMA ring, swizzle and swapped 16x16x32 MFMA step as gemm_core.h, so every
//      accumulator sums its products in the same order as the unfused GEMM;
//   2. epilogue: + bias, round to bf16, written into LDS as the attention core's Q / K / V images (row-major
//      [Tpad][dh + 8] for Q and K, [Tpad][LDV] for V) -- the ring is reused, nothing goes to HBM;
//   3. attention: the waves walk (head, 32-query block) items with the shared core (attn_core.h), O -> HBM.
// Q, K, V and O are bit-identical to the unfused qkv GEMM + mha_fwd_bf16_kernel (tests/test_gpu_kernels.py).
// Rows past T are copies of row T - 1 (clamped DMA rows): masked as keys, never stored as queries.
// One workgroup per CU (8 waves; 88-126 KiB of LDS); workgroups of one image run back to back on one XCD
// (xcd_remap), so its X rows are fetched into that L2 once for all heads.
#include "attn_core.h"
#include "gemm_core.h"

namespace qa {
constexpr int NW = 8, WGN = 4, WGM = 2;  // waves: 4 along the 192 weight columns, 2 along the tokens
// BK = 64: 128-B LDS rows (8 chunks), 2 stages, one workgroup per CU.  BK = 32: 64-B rows (4 chunks), 3 stages
// (counted vmcnt), the rows padded to whole rounds of 16-row pieces so every wave issues the same count; the ring
// then fits beside nothing else but stays under the attention images, so two workgroups share a CU.
template <int DH, int HG, int TPAD, int BK = 64> struct Cfg {
  static constexpr int NC = 3 * HG * DH;            // GEMM columns (weight rows) of the workgroup
  static constexpr int RB = 2 * BK;                 // bytes per LDS row
  static constexpr int PROWS = 1024 / RB;           // rows per 1-KiB LDS-DMA piece
  static constexpr int NS = BK == 64 ? 2 : 3;       // ring stages
  static constexpr int ROWS0 = NC + TPAD;
  static constexpr int ROWS = BK == 64 ? ROWS0 : (ROWS0 + NW * PROWS - 1) / (NW * PROWS) * (NW * PROWS);
  static constexpr int PIECES = ROWS / PROWS;       // LDS-DMA pieces per stage
  static constexpr int PPW = (PIECES + NW - 1) / NW;  // pieces per wave (the last round partial at BK = 64)
  static constexpr int WN = NC / WGN, WM = TPAD / WGM;
  static constexpr int TN = WN / 16, TM = WM / 16;
  static constexpr int LDQ = DH + 8, LDV = AttnTr<DH>::LDV;
  static constexpr int QK_BYTES = TPAD * LDQ * 2, V_BYTES = TPAD * LDV * 2;
  static constexpr int HEAD_BYTES = 2 * QK_BYTES + V_BYTES;  // Q, K, V images of one head
  static constexpr int RING = NS * ROWS * RB;
  static constexpr int LDS = RING > HG * HEAD_BYTES ? RING : HG * HEAD_BYTES;
  static constexpr int WG_PER_CU = BK == 64 ? 1 : 2;
  static_assert(ROWS % 8 == 0 && WN % 16 == 0 && WM % 16 == 0 && TPAD % 32 == 0, "qkv_attn tile");
  static_assert(LDV > 0 && DH % 32 == 0, "qkv_attn: head dim with a lean attention core");
  static_assert(LDS * WG_PER_CU <= 160 * 1024, "qkv_attn: LDS");
  static_assert(BK == 64 || ROWS % (NW * PROWS) == 0, "qkv_attn: BK 32 rows in whole rounds");
};

// 64-B LDS rows: chunk c of row r at slot c ^ (((r >> 3) & 1) << 1) -- the ds_read_b128 fragment reads of 16
// consecutive rows x 4 chunks are conflict-free in all four lane groups
__device__ __forceinline__ int slot32(int r, int c) { return c ^ (((r >> 3) & 1) << 1); }

// one 32-deep K-step of the swapped 16x16x32 MFMA tile over 64-B rows (A = weight rows [0, BN), B = token rows)
template <int BN, int WN, int WM, int TN, int TM>
__device__ __forceinline__ void mfma_tile32(const unsigned char* stage, int wn, int wm, int lane, f32x4 (&acc)[TN][TM]) {
  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 a[TN], b[TM];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int r = wn * WN + 16 * i + fr;
    a[i] = *reinterpret_cast<const bf16x8*>(stage + r * 64 + 16 * slot32(r, fq));
  }
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int r = BN + wm * WM + 16 * j + fr;
    b[j] = *reinterpret_cast<const bf16x8*>(stage + r * 64 + 16 * slot32(r, fq));
  }
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}
}  // namespace qa

template <int DH, int HG, int TPAD, int BK>
__global__ void __launch_bounds__(qa::NW * 64, BK == 64 ? 1 : 2)
qkv_attn_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, const float* __restrict__ bias,
                bf16* __restrict__ out, int T, int H, float scale_log2e) {
  using C = qa::Cfg<DH, HG, TPAD, BK>;
  constexpr int NW = qa::NW, WGN = qa::WGN;
  constexpr int NC = C::NC, TN = C::TN, TM = C::TM, WN = C::WN, WM = C::WM, LDQ = C::LDQ, LDV = C::LDV;
  __shared__ __attribute__((aligned(16))) uint4 lds[C::LDS / 16];

  const int ngroups = H / HG;
  const int item = xcd_remap(blockIdx.x, gridDim.x), b = item / ngroups, g = item - b * ngroups;
  const int D = H * DH, HD = HG * DH;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WGN, wm = wave / WGN;
  const bf16* xb = x + (size_t)b * T * D;

  // ---- 1. GEMM: acc[n][m] = sum_k W[row(n)][k] X[b, m][k]; weight row of column n (q | k | v parts, each the
  // HD rows of this head group): part * D + g * HD + n % HD
  constexpr int LPR = BK / 8;                      // 16-B chunks per LDS row
  const int pch = lane % LPR;
  const bf16* src[C::PPW];
  int swz[C::PPW];
#pragma unroll
  for (int j = 0; j < C::PPW; ++j) {
    const int r = C::PROWS * (wave + NW * j) + lane / LPR;  // LDS row this lane fills
    const int rr = min(r, C::ROWS - 1);
    if (rr < NC) {
      const int part = rr / HD;
      src[j] = w + (size_t)(part * D + g * HD + (rr - part * HD)) * D;
    } else {
      src[j] = xb + (size_t)min(rr - NC, T - 1) * D;  // rows past T (and the BK-32 round padding): the last row
    }
    swz[j] = BK == 64 ? pch ^ ((r >> 1) & 7) : qa::slot32(r, pch);  // source chunk of this lane's LDS slot
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_void_t*)lds;
  const unsigned wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto issue = [&](int stage, int kt) {
    const unsigned sb = lds_base + (unsigned)stage * C::ROWS * C::RB;
#pragma unroll
    for (int j = 0; j < C::PPW; ++j) {
      if (C::PIECES % NW == 0 || (int)wave_u + NW * j < C::PIECES)  // wave-uniform: the last round is partial
        glds16(src[j] + kt * BK + swz[j] * 8, sb + (wave_u + NW * j) * 1024u);
    }
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = D / BK;
  if constexpr (BK == 64) {
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int stage = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) issue(stage ^ 1, kt + 1);
      mfma_tile<bf16, NC, WN, WM, TN, TM>(lds + stage * C::ROWS * 8, wn, wm, lane, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stage ^= 1;
    }
  } else {
    // 3-stage ring: step kt reads stage kt % 3 and issues step kt + 2 into the stage step kt - 1 read (retired by
    // the barrier that closed step kt - 1); counted waits keep the younger stage in flight
    constexpr int PER = C::PPW;
    const unsigned char* lb0 = reinterpret_cast<const unsigned char*>(lds);
    issue(0, 0);
    if (nk > 1) issue(1, 1);
    gemm_ring_wait<PER, 3>(min(1, nk - 1));
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 2 < nk) issue((kt + 2) % 3, kt + 2);
      qa::mfma_tile32<NC, WN, WM, TN, TM>(lb0 + (kt % 3) * C::ROWS * C::RB, wn, wm, lane, acc);
      gemm_ring_wait<PER, 3>(min(kt + 2, nk - 1) - (kt + 1));
    }
  }

  // ---- 2. + bias, bf16, into the per-head Q / K / V images (the ring is free after the last barrier)
  // acc[i][j]: columns n = wn*WN + 16 i + 4 fq + 0..3 (never crossing a head), token m = wm*WM + 16 j + fr
  unsigned char* lb = reinterpret_cast<unsigned char*>(lds);
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = wn * WN + 16 * i + 4 * fq;
    const int part = n / HD, within = n - part * HD, hj = within / DH, d = within - hj * DH;
    const f32x4 bv = load4f(bias + part * D + g * HD + within);
    unsigned char* head = lb + hj * C::HEAD_BYTES;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = wm * WM + 16 * j + fr;
      const f32x4 v = acc[i][j] + bv;
      bf16x4 o;
      o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
      bf16* dst = part == 2 ? reinterpret_cast<bf16*>(head + 2 * C::QK_BYTES) + (size_t)m * LDV + d
                            : reinterpret_cast<bf16*>(head + part * C::QK_BYTES) + (size_t)m * LDQ + d;
      *reinterpret_cast<bf16x4*>(dst) = o;
    }
  }
  __syncthreads();

  // ---- 3. attention: (head, 32-query block) items over the waves
  constexpr int NQB = TPAD / 32;
  for (int it = wave; it < HG * NQB; it += NW) {
    const int hj = it / NQB, q0 = 32 * (it - hj * NQB);
    if (q0 >= T) continue;  // wave-uniform
    const unsigned char* head = lb + hj * C::HEAD_BYTES;
    const bf16* Qs = reinterpret_cast<const bf16*>(head);
    const bf16* Ks = reinterpret_cast<const bf16*>(head + C::QK_BYTES);
    const bf16* Vs = reinterpret_cast<const bf16*>(head + 2 * C::QK_BYTES);
    bf16x8 qf[DH / 16];
    const bf16* qrow = Qs + (size_t)(q0 + (lane & 31)) * LDQ + 8 * (lane >> 5);
#pragma unroll
    for (int s2 = 0; s2 < DH / 16; ++s2) qf[s2] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s2);
    mha_bf16_item<DH>(Ks, Vs, qf, T, TPAD, scale_log2e, lane, q0, nullptr,
                      out + (size_t)b * T * D + (size_t)(g * HG + hj) * DH, D);
  }
}

// ViT-B encoder (T 145): BK 32, two workgroups per CU -- 49.0 vs 51.6 us per launch, forward +2 % same box
// (profiles/r04/c8_*).  K = 64 (T 65): BK 64 (the BK-32 rows padded to whole 128-row rounds add a third: 31.3 vs
// 29.2 us).  A/B builds: tools/build_variant.sh qkv_attn.hip -DTMAE_QA_ENC_BK=64
#ifndef TMAE_QA_ENC_BK
#define TMAE_QA_ENC_BK 32
#endif
template <int DH, int HG, int TPAD, int BK = (DH == 64 && TPAD == 160 ? TMAE_QA_ENC_BK : 64)>
static int qkv_attn_launch(const bf16* x, const bf16* w, const float* b, bf16* out, int B, int T, int H, float scale,
                           hipStream_t st) {
  hipLaunchKernelGGL((qkv_attn_kernel<DH, HG, TPAD, BK>), dim3(B * (H / HG)), dim3(qa::NW * 64), 0, st, x, w, b, out, T,
                     H, scale * 1.4426950408889634f);
  TMAE_LAUNCH_CHECK("tmae_qkv_attn_fwd");
}

// the (head dim, sequence) shapes with a fused instantiation; others take the unfused qkv GEMM + tmae_mha_fwd
static bool qkv_attn_shape(int T, int H, int dh, int& hg, int& tpad) {
  tpad = (T + 31) / 32 * 32;
  if (dh == 64 && tpad == 160) { hg = 1; return true; }                     // ViT-B encoder, K = 144 (T 145)
  if (dh == 64 && tpad == 96) { hg = 1; return true; }                      // ViT-B encoder, K = 64 (T 65)
  if (dh == 32 && tpad == 288 && H % 2 == 0) { hg = 2; return true; }      // decoder 512 / 16 heads (T 257)
  return false;
}

extern "C" int tmae_qkv_attn_supported(int T, int H, int dh) {
  int hg, tpad;
  return T >= 1 && H >= 1 && qkv_attn_shape(T, H, dh, hg, tpad) ? 1 : 0;
}

extern "C" int tmae_qkv_attn_fwd(const void* x, const void* w_qkv, const float* b_qkv, void* out, int B, int T, int H,
                                 int dh, float scale, int dtype, void* stream) {
  TMAE_REQUIRE(dtype == TMAE_BF16, "tmae_qkv_attn_fwd: bf16 operands only (the f32 path runs unfused)");
  TMAE_REQUIRE(x && w_qkv && b_qkv && out, "tmae_qkv_attn_fwd: null pointer");
  TMAE_REQUIRE(B >= 0 && T >= 1 && H >= 1, "tmae_qkv_attn_fwd: B=%d T=%d H=%d", B, T, H);
  TMAE_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)w_qkv & 15) == 0 && ((uintptr_t)b_qkv & 15) == 0 &&
               ((uintptr_t)out & 7) == 0, "tmae_qkv_attn_fwd: misaligned operand");
  int hg, tpad;
  TMAE_REQUIRE(qkv_attn_shape(T, H, dh, hg, tpad), "tmae_qkv_attn_fwd: no fused kernel for T=%d, %d heads of dim %d",
               T, H, dh);
  if (B == 0) return TMAE_OK;
  hipStream_t st = (hipStream_t)stream;
  const bf16* xp = (const bf16*)x;
  const bf16* wp = (const bf16*)w_qkv;
  bf16* op = (bf16*)out;
  if (dh == 64 && tpad == 160) return qkv_attn_launch<64, 1, 160>(xp, wp, b_qkv, op, B, T, H, scale, st);
  if (dh == 64 && tpad == 96) return qkv_attn_launch<64, 1, 96>(xp, wp, b_qkv, op, B, T, H, scale, st);
  return qkv_attn_launch<32, 2, 288>(xp, wp, b_qkv, op, B, T, H, scale, st);
}
