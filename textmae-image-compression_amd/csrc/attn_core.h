// Shared bf16 attention core (timm Attention, MCM.py:629-630, 678-679): one wave's 32 queries against K / V
// of one (image, head) staged in LDS.  Used by the standalone attention kernel (attention.hip) and by the
// fused qkv-GEMM + attention kernel (qkv_attn.hip), so both compute bit-identical outputs.
#pragma once

#include "common.h"

// bf16 forward, VALU-lean form of the plain kernel in attention.hip (the softmax VALU, not the MFMA pipe, bounds the loop:
// a 32-key tile costs DH/16 + DH/16 MFMAs against 16 scores of exp/max/sum per lane):
//   * the scale rides in the exponent: p = exp2(s * c - m * c) is one FMA + v_exp, no per-score multiply;
//   * masking only on the ragged last key tile (wave-uniform branch);
//   * deferred rescaling (cdna_hip_programming.md T13): the running max m only moves when some lane's tile
//     max exceeds it by more than 8 (log2 units), so O / l are rescaled on the first tile and rarely after;
//     P <= 2^8, exact after the final 1/l (same m for O and l);
//   * per-lane partial row sums, combined across the two lane halves once at the end;
//   * V^T staged with keys on consecutive lanes (2-byte LDS stores to consecutive addresses).
template <int DH> struct AttnTr { static constexpr int LDV = 0; };  // no lean form
// V row stride (elements) for conflict-free ds_read_b64_tr_b16: 4 key rows x 2 lane groups of 8 dwords
// must cover all 64 banks -> row stride = 16 or 48 dwords mod 64
template <> struct AttnTr<64> { static constexpr int LDV = 96; };
template <> struct AttnTr<32> { static constexpr int LDV = 32; };

typedef __attribute__((ext_vector_type(4))) short attn_s4;
typedef __attribute__((address_space(3))) attn_s4 attn_lds_s4;

typedef __attribute__((ext_vector_type(2))) float attn_f2;

// max / sum over the two lane halves (lane l <-> l ^ 32) without an LDS round trip: v_permlane32_swap with
// the value in both operands returns {own, partner} in lanes 0-31 and {partner, own} in lanes 32-63
__device__ __forceinline__ float attn_xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float attn_xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// one (image, head) item of the bf16 forward: this wave's 32 queries against the K / V tiles staged in
// LDS (Ks row-major [Tpad][DH + 8], Vs row-major [Tpad][LDV]); writes O (and the base-2 LSE when lse).
// Software pipeline: the S^T MFMAs of key tile kt+1 are issued before the softmax of tile kt, so they run
// under its VALU work instead of stalling the max reduction.  The softmax runs on packed pairs
// (v_pk_fma_f32 / v_pk_add_f32), the cross-half reductions on v_permlane32_swap, and only the last key
// tile carries the ragged-length mask (peeled out of the loop).
template <int DH>
__device__ __forceinline__ void mha_bf16_item(const bf16* Ks, const bf16* Vs, const bf16x8 (&qf)[DH / 16], int Tn,
                                              int Tpad, float scale_log2e, int lane, int q0, float* lse, bf16* obase,
                                              int D) {
  constexpr int KPAD = 8, NDT = DH / 32, LDV = AttnTr<DH>::LDV;
  constexpr int ldk = DH + KPAD;
  const int col = lane & 31, hh = lane >> 5;
  const int q = q0 + col;
  // transposed-read lane roles: group g = lane >> 4 reads keys k0 + 4*(g>>1) + qq, d columns 16*(g&1) + 4*pp
  const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
  const int trow = 4 * (g >> 1) + qq, tcol = 16 * (g & 1) + 4 * pp;

  f32x16 O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[dt][r] = 0.0f;
  const float c = scale_log2e;
  const float thr = 8.0f / c;  // 8 in log2 units, in raw-score units
  float m_run = -INFINITY;
  attn_f2 l2 = {0.0f, 0.0f};
  const int ntiles = Tpad / 32;
  const bool ragged = (Tn & 31) != 0;

  auto qk = [&](int kt) {
    f32x16 S;
#pragma unroll
    for (int r = 0; r < 16; ++r) S[r] = 0.0f;
    const bf16* krow = Ks + (size_t)(32 * kt + col) * ldk + 8 * hh;
#pragma unroll
    for (int s2 = 0; s2 < DH / 16; ++s2) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(krow + 16 * s2);
      S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s2], S, 0, 0, 0);
    }
    return S;
  };
  auto step = [&](f32x16 S, int kt, bool mask) {
    if (mask) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (key >= Tn) S[r] = -INFINITY;
      }
    }
    float t0 = fmaxf(fmaxf(S[0], S[1]), S[2]), t1 = fmaxf(fmaxf(S[3], S[4]), S[5]);
    float t2 = fmaxf(fmaxf(S[6], S[7]), S[8]), t3 = fmaxf(fmaxf(S[9], S[10]), S[11]);
    float t4 = fmaxf(fmaxf(S[12], S[13]), S[14]);
    const float tmax = attn_xhalf_max(fmaxf(fmaxf(fmaxf(t0, t1), fmaxf(t2, t3)), fmaxf(t4, S[15])));
    const bool grow = tmax > m_run + thr;
    if (__builtin_amdgcn_ballot_w64(grow)) {
      const float m_new = grow ? tmax : m_run;
      const float alpha = exp2f((m_run - m_new) * c);
      l2 *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[dt] *= alpha;
      m_run = m_new;
    }
    const attn_f2 c2 = {c, c}, mc2 = {-m_run * c, -m_run * c};
    float P[16];
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      const attn_f2 e = __builtin_elementwise_fma((attn_f2){S[r], S[r + 1]}, c2, mc2);
      const attn_f2 p = {__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
      l2 += p;
      P[r] = p.x;
      P[r + 1] = p.y;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = (bf16)P[8 * s2 + j];
      const int k0 = 32 * kt + 16 * s2;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        // A operand = V^T rows (d) x keys k0 + 8(j>>2) + 4hh + (j&3): two 4-key transposed reads
        const bf16* vp = Vs + (size_t)(k0 + trow) * LDV + 32 * dt + tcol;
        const attn_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((attn_lds_s4*)vp);
        const attn_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((attn_lds_s4*)(vp + 8 * LDV));
        typedef __attribute__((ext_vector_type(8))) short s8;
        s8 av;
        av[0] = lo[0]; av[1] = lo[1]; av[2] = lo[2]; av[3] = lo[3];
        av[4] = hi[0]; av[5] = hi[1]; av[6] = hi[2]; av[7] = hi[3];
        O[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<bf16x8*>(&av), pb, O[dt], 0, 0, 0);
      }
    }
  };
  // two tiles per trip so the look-ahead scores alternate between two register sets (no copies)
  f32x16 S0 = qk(0);
  int kt = 0;
  for (; kt + 2 < ntiles; kt += 2) {
    const f32x16 S1 = qk(kt + 1);
    step(S0, kt, false);
    S0 = qk(kt + 2);
    step(S1, kt + 1, false);
  }
  if (kt + 1 < ntiles) {
    const f32x16 S1 = qk(kt + 1);
    step(S0, kt, false);
    step(S1, kt + 1, ragged);
  } else {
    step(S0, kt, ragged);
  }
  const float l_run = attn_xhalf_sum(l2.x + l2.y);
  if (q >= Tn) return;
  if (lse && hh == 0) lse[q] = m_run * c + log2f(l_run);
  const float inv_l = 1.0f / l_run;
  bf16* orow = obase + (size_t)q * D;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      const int d = 32 * dt + 8 * gg + 4 * hh;
      f32x4 v{O[dt][4 * gg] * inv_l, O[dt][4 * gg + 1] * inv_l, O[dt][4 * gg + 2] * inv_l, O[dt][4 * gg + 3] * inv_l};
      store4(orow + d, v);
    }
}
