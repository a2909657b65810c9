// Fused multi-head self-attention for the ViT encoder / decoder blocks (timm 0.4.5 Attention:
// softmax((q @ k^T) * dh^-0.5) @ v, called from MCM.py:629-630, 678-679).
//
// Sequences are short (T = K+1 = 145 in the encoder, L+1 = 257 in the decoder), so one workgroup
// owns one (image, head): it stages K (row-major) and V (transposed) of that head in LDS ONCE and
// every wave of the workgroup walks 32 queries against them.  Per wave and 32-key tile:
//   S^T = K_tile · Q^T      (v_mfma_f32_32x32x16_bf16 / 32x32x2_f32): each lane holds 16 of the
//                           32 scores of ONE query -> the softmax row max/sum is 16 register ops
//                           plus one cross-half shuffle, no LDS
//   O^T += V^T · P^T        the score accumulator is fed straight back as the MFMA B operand
//                           (cdna_hip_programming.md §3 "accumulator tile as the next operand")
// Online (flash) softmax over key tiles; the [T x T] score matrix never exists in HBM.
#include <stdlib.h>

#include "attn_core.h"

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16> { static constexpr int KPAD = 8, VPAD = 4, EPC = 8; };
template <> struct AttnCfg<float> { static constexpr int KPAD = 4, VPAD = 1, EPC = 4; };

// MAXT: the launch bound (the dh-80 / ViT-H case also has a 512-thread instance: at 1024 it spilled 3 VGPRs)
template <typename T, int DH, int MAXT = 1024>
__global__ void __launch_bounds__(MAXT)
mha_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ out, float* __restrict__ lse, int Tn, int H, int Tpad,
               float scale_log2e) {
  constexpr int KPAD = AttnCfg<T>::KPAD, VPAD = AttnCfg<T>::VPAD, EPC = AttnCfg<T>::EPC;
  // 32-wide output tiles along the head dim; a head dim that is not a multiple of 32 (ViT-H: 80) gets
  // zero rows DH..DHP-1 in V^T, so the last tile's extra output columns are zero and never stored
  constexpr int DHP = (DH + 31) / 32 * 32, NDT = DHP / 32;
  static_assert(DH % 16 == 0, "head dim must be a multiple of 16");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldk = DH + KPAD, ldv = Tpad + VPAD;
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vt = Ks + (size_t)Tpad * ldk;

  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const T* base = qkv + (size_t)b * Tn * ld + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;

  // stage K [Tpad][DH] and V^T [DHP][Tpad] of this head
  constexpr int CPR = DH / EPC;  // 16-B chunks per row
  if constexpr (DHP != DH)
    for (int i = tid; i < (DHP - DH) * ldv; i += nthr) Vt[(size_t)DH * ldv + i] = (T)0.0f;
  for (int i = tid; i < Tpad * CPR; i += nthr) {
    const int r = i / CPR, c = i - r * CPR;
    uint4 kv = uint4{0, 0, 0, 0}, vv = uint4{0, 0, 0, 0};
    if (r < Tn) {
      kv = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + D + c * EPC);
      vv = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + 2 * D + c * EPC);
    }
    *reinterpret_cast<uint4*>(Ks + (size_t)r * ldk + c * EPC) = kv;
    const T* ve = reinterpret_cast<const T*>(&vv);
#pragma unroll
    for (int e = 0; e < EPC; ++e) Vt[(size_t)(c * EPC + e) * ldv + r] = ve[e];
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6;
  const int q0 = wave * 32;
  if (q0 >= Tn) return;
  const int col = lane & 31, hh = lane >> 5;
  const int q = q0 + col;
  const int qc = q < Tn ? q : Tn - 1;
  const T* qrow = base + (size_t)qc * ld;

  f32x16 O[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) O[dt][r] = 0.0f;
  float m_run = -INFINITY, l_run = 0.0f;

  const int ntiles = Tpad / 32;
  if constexpr (sizeof(T) == 2) {
    bf16x8 qf[DH / 16];
#pragma unroll
    for (int s = 0; s < DH / 16; ++s) qf[s] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s + 8 * hh);
    for (int kt = 0; kt < ntiles; ++kt) {
      f32x16 S;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = 0.0f;
      const T* krow = Ks + (size_t)(32 * kt + col) * ldk + 8 * hh;
#pragma unroll
      for (int s = 0; s < DH / 16; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(krow + 16 * s);
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], S, 0, 0, 0);
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
        S[r] = (key < Tn) ? S[r] * scale_log2e : -INFINITY;
        tmax = fmaxf(tmax, S[r]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = exp2f(m_run - m_new);
      float ps = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        S[r] = exp2f(S[r] - m_new);
        ps += S[r];
      }
      ps += __shfl_xor(ps, 32);
      l_run = l_run * alpha + ps;
      m_run = m_new;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[dt] *= alpha;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (bf16)S[8 * s + j];
        const int k0 = 32 * kt + 16 * s + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const T* vrow = Vt + (size_t)(32 * dt + col) * ldv + k0;
          const bf16x4 v0 = *reinterpret_cast<const bf16x4*>(vrow);
          const bf16x4 v1 = *reinterpret_cast<const bf16x4*>(vrow + 8);
          bf16x8 a;
          a[0] = v0[0]; a[1] = v0[1]; a[2] = v0[2]; a[3] = v0[3];
          a[4] = v1[0]; a[5] = v1[1]; a[6] = v1[2]; a[7] = v1[3];
          O[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, pb, O[dt], 0, 0, 0);
        }
      }
    }
  } else {
    float qf[DH / 2];
#pragma unroll
    for (int s = 0; s < DH / 2; ++s) qf[s] = qrow[2 * s + hh];
    for (int kt = 0; kt < ntiles; ++kt) {
      f32x16 S;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = 0.0f;
      const T* krow = Ks + (size_t)(32 * kt + col) * ldk + hh;
#pragma unroll
      for (int s = 0; s < DH / 2; ++s) S = __builtin_amdgcn_mfma_f32_32x32x2f32(krow[2 * s], qf[s], S, 0, 0, 0);
      float tmax = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
        S[r] = (key < Tn) ? S[r] * scale_log2e : -INFINITY;
        tmax = fmaxf(tmax, S[r]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32));
      const float m_new = fmaxf(m_run, tmax);
      const float alpha = exp2f(m_run - m_new);
      float ps = 0.0f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        S[r] = exp2f(S[r] - m_new);
        ps += S[r];
      }
      ps += __shfl_xor(ps, 32);
      l_run = l_run * alpha + ps;
      m_run = m_new;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) O[dt] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = 32 * kt + (r & 3) + 8 * (r >> 2) + 4 * hh;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const float a = Vt[(size_t)(32 * dt + col) * ldv + key];
          O[dt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, S[r], O[dt], 0, 0, 0);
        }
      }
    }
  }

  if (q >= Tn) return;
  if (lse && hh == 0) lse[(size_t)bh * Tn + q] = m_run + log2f(l_run);  // base-2 log-sum-exp of the scaled scores
  const float inv_l = 1.0f / l_run;
  T* orow = out + ((size_t)b * Tn + q) * D + h * DH;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hh;
      if (DHP != DH && d >= DH) continue;
      f32x4 v{O[dt][4 * g] * inv_l, O[dt][4 * g + 1] * inv_l, O[dt][4 * g + 2] * inv_l, O[dt][4 * g + 3] * inv_l};
      store4(orow + d, v);
    }
}

// one workgroup per (image, head): K / V staged in LDS, one 32-query block per wave.  Workgroup ids go
// through xcd_remap, so the heads of one image run back to back on one XCD: at dh = 32 two heads share every
// 128-B line of qkv, which one L2 then fetches once instead of each of two XCDs fetching it.
template <int DH>
__global__ void __launch_bounds__(1024)
mha_fwd_bf16_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, float* __restrict__ lse, int Tn, int H,
                    int Tpad, float scale_log2e) {
  constexpr int KPAD = 8, CPR = DH / 8, LDV = AttnTr<DH>::LDV;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int ldk = DH + KPAD;
  bf16* Ks = reinterpret_cast<bf16*>(smem);
  bf16* Vs = Ks + (size_t)Tpad * ldk;
  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const bf16* base = qkv + (size_t)b * Tn * ld + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;
  // K and V row-major, 16-B chunks; every load of a thread issued before its first LDS store
  // chunks per thread per operand: Tpad * DH / 8 chunks over >= 2 * Tpad threads
  constexpr int MAXC = DH / 16;
  uint4 kv[MAXC], vv[MAXC];
#pragma unroll
  for (int u = 0; u < MAXC; ++u) {
    const int i = tid + u * nthr;
    const int r = i / CPR, c = i - r * CPR;
    kv[u] = vv[u] = uint4{0, 0, 0, 0};
    if (r < Tn && i < Tpad * CPR) {
      kv[u] = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + D + c * 8);
      vv[u] = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + 2 * D + c * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < MAXC; ++u) {
    const int i = tid + u * nthr;
    if (i < Tpad * CPR) {
      const int r = i / CPR, c = i - r * CPR;
      *reinterpret_cast<uint4*>(Ks + (size_t)r * ldk + c * 8) = kv[u];
      *reinterpret_cast<uint4*>(Vs + (size_t)r * LDV + c * 8) = vv[u];
    }
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6;
  const int q0 = wave * 32;
  if (q0 >= Tn) return;  // whole wave: EXEC stays all-ones for the transposed reads below
  // (Q issued with the K / V loads instead, one HBM round trip for both, measured 5-10 % slower)
  const bf16* qrow = base + (size_t)min(q0 + (lane & 31), Tn - 1) * ld;
  bf16x8 qf[DH / 16];
#pragma unroll
  for (int s2 = 0; s2 < DH / 16; ++s2) qf[s2] = *reinterpret_cast<const bf16x8*>(qrow + 16 * s2 + 8 * (lane >> 5));
  mha_bf16_item<DH>(Ks, Vs, qf, Tn, Tpad, scale_log2e, lane, q0, lse ? lse + (size_t)bh * Tn : nullptr,
                    out + (size_t)b * Tn * D + h * DH, D);
}

template <typename T, int DH>
static int mha_launch(const void* qkv, void* out, int B, int Tn, int H, float scale, hipStream_t st,
                      float* lse = nullptr) {
  const int Tpad = (Tn + 31) / 32 * 32;
  constexpr bool lean_ok = sizeof(T) == 2 && DH % 32 == 0;  // the VALU-lean kernel takes whole 32-wide tiles
  constexpr int DHP = (DH + 31) / 32 * 32;
  const bool lean = lean_ok;  // the plain kernel: f32 and the ViT-H head dim 80 (lean: 18 vs 23 us enc, 30 vs 44 dec)
  const int nthr = 64 * (Tpad / 32);
  const size_t lds = lean ? ((size_t)Tpad * (DH + 8) + (size_t)Tpad * AttnTr<DH>::LDV) * 2
                          : ((size_t)Tpad * (DH + AttnCfg<T>::KPAD) + (size_t)DHP * (Tpad + AttnCfg<T>::VPAD)) * sizeof(T);
  TMAE_REQUIRE(nthr <= 1024 && lds <= 160 * 1024, "tmae_mha_fwd: sequence length %d too long", Tn);
  TMAE_REQUIRE(!lean || Tpad * (DH / 8) <= nthr * (DH / 16), "tmae_mha_fwd: sequence length %d too long", Tn);
  if (B * H == 0 || Tn == 0) return TMAE_OK;
  if constexpr (lean_ok) {
    if (lean) {
      hipLaunchKernelGGL((mha_fwd_bf16_kernel<DH>), dim3(B * H), dim3(nthr), lds, st, (const bf16*)qkv, (bf16*)out,
                         lse, Tn, H, Tpad, scale * 1.4426950408889634f);
      TMAE_LAUNCH_CHECK("tmae_mha_fwd");
    }
  }
  constexpr int M80 = (DH == 80 && sizeof(T) == 2) ? 512 : 1024;  // the 512-bound instance: bf16 dh 80 only
  if (M80 == 512 && nthr <= 512)
    hipLaunchKernelGGL((mha_fwd_kernel<T, DH, M80>), dim3(B * H), dim3(nthr), lds, st, (const T*)qkv, (T*)out, lse, Tn,
                       H, Tpad, scale * 1.4426950408889634f);
  else
    hipLaunchKernelGGL((mha_fwd_kernel<T, DH>), dim3(B * H), dim3(nthr), lds, st, (const T*)qkv, (T*)out, lse, Tn, H,
                       Tpad, scale * 1.4426950408889634f);
  TMAE_LAUNCH_CHECK("tmae_mha_fwd");
}

template <typename E>
static int mha_dispatch(const void* qkv, void* out, int B, int T, int H, int dh, float scale, hipStream_t st,
                        float* lse) {
  if (dh == 64) return mha_launch<E, 64>(qkv, out, B, T, H, scale, st, lse);
  if (dh == 80) return mha_launch<E, 80>(qkv, out, B, T, H, scale, st, lse);  // ViT-H (models_mae.py:239-244)
  return mha_launch<E, 32>(qkv, out, B, T, H, scale, st, lse);
}

extern "C" int tmae_mha_fwd(const void* qkv, void* out, int B, int T, int H, int dh, float scale, int dtype,
                            void* stream) {
  TMAE_REQUIRE(dh == 32 || dh == 64 || dh == 80, "tmae_mha_fwd: head dim %d unsupported (32, 64 or 80)", dh);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16) return mha_dispatch<bf16>(qkv, out, B, T, H, dh, scale, st, nullptr);
  return mha_dispatch<float>(qkv, out, B, T, H, dh, scale, st, nullptr);
}

extern "C" int tmae_mha_fwd_lse(const void* qkv, void* out, float* lse, int B, int T, int H, int dh, float scale,
                                int dtype, void* stream) {
  TMAE_REQUIRE(dh == 32 || dh == 64 || dh == 80, "tmae_mha_fwd_lse: head dim %d unsupported (32, 64 or 80)", dh);
  TMAE_REQUIRE(lse != nullptr, "tmae_mha_fwd_lse: lse is NULL");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16) return mha_dispatch<bf16>(qkv, out, B, T, H, dh, scale, st, lse);
  return mha_dispatch<float>(qkv, out, B, T, H, dh, scale, st, lse);
}

// ====================================================================================== backward
// Flash-style attention backward (timm Attention, MCM.py:629-630, 678-679): P is recomputed from Q, K and
// the forward's base-2 log-sum-exp; one workgroup owns one (image, head) and holds Q, K, V, dO (row-major)
// plus Q^T, K^T, dO^T in LDS for the whole sequence.
//   phase 1 (wave = 32 keys, loop over query tiles):  S = Q K^T, dP = dO V^T with the key on the lane, so
//            P and dS = P (dP - delta) are already the A operands of dV += P^T dO and dK += scale dS^T Q
//            (cdna_hip_programming.md §3, "accumulator tile as the next operand");
//   phase 2 (wave = 32 queries, loop over key tiles): S^T, dP^T with the query on the lane -> dQ += scale dS K.
// Both phases own their outputs: no atomics, bitwise reproducible.  delta = rowsum(dO * O).
template <int DH> struct AttnBwd;
// LDS row stride (elements) of the staged operands: both row-wise ds_read_b128 fragment reads and
// ds_read_b64_tr_b16 transposed reads come from the same rows; 48 / 16 dwords keep the transposed reads
// conflict-free (as the forward's V^T)
template <> struct AttnBwd<64> { static constexpr int LDR = 96; };
template <> struct AttnBwd<32> { static constexpr int LDR = 32; };
template <> struct AttnBwd<80> { static constexpr int LDR = 96; };  // columns 80..95 staged as zeros

// B (or A) operand of a 32x32x16 MFMA whose k runs over 16 ROWS of a row-major LDS array (rows k0.., the
// 32 columns c0..c0+31 on the lanes): two transposed 4-row reads, the element order of the accumulator
// layout (k = (j & 3) + 8 (j >> 2) + 4 hh), as the forward's V^T operand
template <int LD>
__device__ __forceinline__ bf16x8 attn_tr_frag(const bf16* arr, int k0, int c0, int lane) {
  const int g = lane >> 4, gi = lane & 15, qq = gi >> 2, pp = gi & 3;
  const int trow = 4 * (g >> 1) + qq, tcol = 16 * (g & 1) + 4 * pp;
  const bf16* p = arr + (size_t)(k0 + trow) * LD + c0 + tcol;
  const attn_s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((attn_lds_s4*)p);
  const attn_s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((attn_lds_s4*)(p + 8 * LD));
  typedef __attribute__((ext_vector_type(8))) short s8;
  s8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return *reinterpret_cast<bf16x8*>(&v);
}

// rows [0, Tpad) of two head slices (row-major, 16-B chunks, zero past Tn and in the columns DH..DHP-1 that
// pad the head dim to whole 32-wide tiles) -> A0 / A1 (stride LDR)
template <int DH, int LDR>
__device__ __forceinline__ void attn_stage2(bf16* A0, const bf16* g0, int ld0, bf16* A1, const bf16* g1, int ld1,
                                            int Tn, int Tpad, int tid, int nthr) {
  constexpr int CPR = (DH + 31) / 32 * 32 / 8;
  for (int i = tid; i < Tpad * CPR; i += nthr) {
    const int r = i / CPR, c = i - r * CPR;
    uint4 x = uint4{0, 0, 0, 0}, y = x;
    if (r < Tn && 8 * c < DH) {
      x = *reinterpret_cast<const uint4*>(g0 + (size_t)r * ld0 + c * 8);
      y = *reinterpret_cast<const uint4*>(g1 + (size_t)r * ld1 + c * 8);
    }
    *reinterpret_cast<uint4*>(A0 + (size_t)r * LDR + c * 8) = x;
    *reinterpret_cast<uint4*>(A1 + (size_t)r * LDR + c * 8) = y;
  }
}

// Two phases over ONE pair of staged arrays (48 / 37 KB instead of the seven arrays of both phases at once,
// so 2-3 workgroups share a CU): phase 1 stages Q and dO (all queries) and reads this wave's 32 keys of K / V
// from global; phase 2 re-stages K and V (all keys) and reads this wave's 32 queries of Q / dO from global.
// The transposed operands (dO^T, Q^T, K^T) are ds_read_b64_tr_b16 reads of the same row-major arrays.
// (dh 32 capped at 96 VGPRs, five waves per SIMD, so that two 9-wave workgroups share a CU: 17 VGPRs spilled
// and the decoder backward went 133 -> 147 us per launch, profiles/r04/c3_at_*.log; not kept)
template <int DH>
__global__ void __launch_bounds__(DH == 32 ? 1024 : 512)  // dh 64 / 80: <= 256 keys, 256 VGPRs
mha_bwd_bf16_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
                    const float* __restrict__ lse, bf16* __restrict__ dqkv, int Tn, int H, int Tpad, float scale) {
  constexpr int LDR = AttnBwd<DH>::LDR;
  constexpr int NDT = (DH + 31) / 32;  // output tiles; columns >= DH of the last one are zero, never stored
  constexpr int CPR = DH / 8;
  static_assert(DH % 16 == 0, "head dim must be a multiple of 16");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16* A0 = reinterpret_cast<bf16*>(smem);
  bf16* A1 = A0 + (size_t)Tpad * LDR;
  float* lse_s = reinterpret_cast<float*>(A1 + (size_t)Tpad * LDR);
  float* dl_s = lse_s + Tpad;

  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const bf16* base = qkv + (size_t)b * Tn * ld + h * DH;
  const bf16* obase = o + (size_t)b * Tn * D + h * DH;
  const bf16* gbase = dout + (size_t)b * Tn * D + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;

  attn_stage2<DH, LDR>(A0, base, ld, A1, gbase, D, Tn, Tpad, tid, nthr);  // Q, dO
  // delta = rowsum(dO * O) (16-B loads, CPR chunks per row), lse
  for (int r = tid; r < Tpad; r += nthr) {
    float d = 0.0f, l = 0.0f;
    if (r < Tn) {
      const bf16* orow = obase + (size_t)r * D;
      const bf16* grow = gbase + (size_t)r * D;
#pragma unroll
      for (int c = 0; c < CPR; ++c) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(orow + 8 * c);
        const bf16x8 gv = *reinterpret_cast<const bf16x8*>(grow + 8 * c);
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)ov[e] * (float)gv[e];
      }
      l = lse[(size_t)bh * Tn + r];
    }
    dl_s[r] = d;
    lse_s[r] = l;
  }
  __syncthreads();

  const int lane = tid & 63, wave = tid >> 6, nw = Tpad / 32;
  const int col = lane & 31, hh = lane >> 5;
  const float c2 = scale * 1.4426950408889634f;
  const bool active = wave < nw;

  // ---------------- phase 1: this wave's 32 keys (K / V rows from global), all queries from LDS
  if (active) {
    const int kb = 32 * wave;
    const int kr = min(kb + col, Tn - 1);
    bf16x8 kf[DH / 16], vf[DH / 16];
#pragma unroll
    for (int s = 0; s < DH / 16; ++s) {
      kf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kr * ld + D + 16 * s + 8 * hh);
      vf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kr * ld + 2 * D + 16 * s + 8 * hh);
    }
    f32x16 dV[NDT], dK[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dV[t][r] = dK[t][r] = 0.0f;
    const bool kok = kb + col < Tn;
    for (int qt = 0; qt < nw; ++qt) {
      f32x16 S, G;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = G[r] = 0.0f;
#pragma unroll
      for (int s = 0; s < DH / 16; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A0 + (size_t)(qt * 32 + col) * LDR + 16 * s + 8 * hh);
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, kf[s], S, 0, 0, 0);
        const bf16x8 g = *reinterpret_cast<const bf16x8*>(A1 + (size_t)(qt * 32 + col) * LDR + 16 * s + 8 * hh);
        G = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g, vf[s], G, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float p = (kok && q < Tn) ? exp2f(S[r] * c2 - lse_s[q]) : 0.0f;
        S[r] = p;
        G[r] = p * (G[r] - dl_s[q]) * scale;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pa, da;
#pragma unroll
        for (int j = 0; j < 8; ++j) { pa[j] = (bf16)S[8 * s + j]; da[j] = (bf16)G[8 * s + j]; }
        const int k0 = qt * 32 + 16 * s;
#pragma unroll
        for (int t = 0; t < NDT; ++t) {
          dV[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, attn_tr_frag<LDR>(A1, k0, 32 * t, lane), dV[t], 0, 0, 0);
          dK[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, attn_tr_frag<LDR>(A0, k0, 32 * t, lane), dK[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (key < Tn && 32 * t + col < DH) {
          bf16* row = dqkv + ((size_t)b * Tn + key) * ld + h * DH + 32 * t + col;
          row[D] = (bf16)dK[t][r];
          row[2 * D] = (bf16)dV[t][r];
        }
      }
  }
  __syncthreads();  // every wave is done with Q / dO in LDS
  attn_stage2<DH, LDR>(A0, base + D, ld, A1, base + 2 * D, ld, Tn, Tpad, tid, nthr);  // K, V
  __syncthreads();

  // ---------------- phase 2: this wave's 32 queries (Q / dO rows from global), all keys from LDS
  if (active) {
    const int qb = 32 * wave;
    const int qr = min(qb + col, Tn - 1);
    bf16x8 qf[DH / 16], gf[DH / 16];
#pragma unroll
    for (int s = 0; s < DH / 16; ++s) {
      qf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)qr * ld + 16 * s + 8 * hh);
      gf[s] = *reinterpret_cast<const bf16x8*>(gbase + (size_t)qr * D + 16 * s + 8 * hh);
    }
    const bool qok = qb + col < Tn;
    const float lq = lse_s[qb + col], dq = dl_s[qb + col];
    f32x16 dQ[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dQ[t][r] = 0.0f;
    for (int kt = 0; kt < nw; ++kt) {
      f32x16 S, G;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = G[r] = 0.0f;
#pragma unroll
      for (int s = 0; s < DH / 16; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(A0 + (size_t)(kt * 32 + col) * LDR + 16 * s + 8 * hh);
        S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, qf[s], S, 0, 0, 0);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(A1 + (size_t)(kt * 32 + col) * LDR + 16 * s + 8 * hh);
        G = __builtin_amdgcn_mfma_f32_32x32x16_bf16(v, gf[s], G, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float p = (qok && key < Tn) ? exp2f(S[r] * c2 - lq) : 0.0f;
        G[r] = p * (G[r] - dq) * scale;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 da;
#pragma unroll
        for (int j = 0; j < 8; ++j) da[j] = (bf16)G[8 * s + j];
        const int k0 = kt * 32 + 16 * s;
#pragma unroll
        for (int t = 0; t < NDT; ++t)
          dQ[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, attn_tr_frag<LDR>(A0, k0, 32 * t, lane), dQ[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (q < Tn && 32 * t + col < DH) dqkv[((size_t)b * Tn + q) * ld + h * DH + 32 * t + col] = (bf16)dQ[t][r];
      }
  }
}

#ifndef TMAE_ATTN_TRACE
#define TMAE_ATTN_TRACE 0  // timeline builds (tools/attn_trace.py): wave 0's shader clock at the backward's phases
#endif
#if TMAE_ATTN_TRACE
// [workgroup][16]: 0 start, 1 prologue barrier passed, 2 + it: step it's barrier passed (<= 10 steps), 14 dK / dV
// stored, 15 dQ stored
static __device__ unsigned long long g_attn_trace[4096 * 16];
#define ATTN_TR(slot)                                                                                          \
  do {                                                                                                         \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_attn_trace[blockIdx.x * 16 + (slot)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
extern "C" int tmae_attn_trace_read(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_attn_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#else
#define ATTN_TR(slot) ((void)0)
#endif

// One-pass form: each wave owns 32 keys (dK^T, dV^T in registers) and walks the query tiles in a STAGGERED order --
// wave w takes tile (w + it) mod nw at step it -- so at every step each query tile belongs to exactly one wave.
// That wave's dQ contribution dS K (dS through a per-wave LDS scratch, the only operand crossing lanes) is added
// into the tile's f32 accumulator in LDS, one barrier per step; every tile receives the waves' contributions in a
// fixed order (bitwise reproducible), and nothing is recomputed: the two-phase form above computed S and dP twice
// (the exp and dS VALU of phase 2) and restaged K / V.  LDS: Q, dO, K [Tpad][LDR] bf16, dS 32 x 32 bf16 per wave,
// dQ [DH][Tpad + 4] f32 (row stride 4 mod 32 dwords: the 16-B read-modify-writes of a half-wave hit 64 banks).
// MAXT: the launch bound.  dh 32 up to 512 threads (<= 256 keys: two workgroups per CU at 128 VGPRs) and from 11
// waves on takes 1024; 9-10 waves (the MCM decoder's 257 tokens) run one workgroup per CU (> 80 KB of LDS), so that
// instance is bounded at 640 threads -> 3 waves per SIMD, 168 VGPRs (at 128 it spilled 10 VGPRs to scratch)
template <int DH, int MAXT = (DH == 32 ? 1024 : 512)>
__global__ void __launch_bounds__(MAXT)  // dh 64: <= 256 keys, up to 256 VGPRs
mha_bwd1_bf16_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ o, const bf16* __restrict__ dout,
                     const float* __restrict__ lse, bf16* __restrict__ dqkv, int Tn, int H, int Tpad, float scale) {
  constexpr int LDR = AttnBwd<DH>::LDR;
  constexpr int NDT = (DH + 31) / 32;
  constexpr int CPR = DH / 8;
  // dh 32: a wave's 32 keys of K ([32][32] bf16, the size of its dS scratch) are staged through that scratch once
  // and held in registers as the dQ product's B fragments, so K takes no LDS of its own (88 -> 74 KB at 224
  // tokens: two workgroups per CU)
  constexpr bool KREG = DH == 32;
  static_assert(DH % 32 == 0, "one-pass backward: whole 32-wide head-dim tiles");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int nw = Tpad / 32, LDQ = Tpad + 4;
  bf16* Qs = reinterpret_cast<bf16*>(smem);
  bf16* Gs = Qs + (size_t)Tpad * LDR;
  bf16* Ks = Gs + (size_t)Tpad * LDR;                      // (not allocated when KREG)
  bf16* dSs = Ks + (KREG ? 0 : (size_t)Tpad * LDR);        // nw x [32 keys][32 queries]
  float* dQs = reinterpret_cast<float*>(dSs + (size_t)nw * 1024);  // [DH][LDQ]
  float* lse_s = dQs + (size_t)DH * LDQ;
  float* dl_s = lse_s + Tpad;

  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const bf16* base = qkv + (size_t)b * Tn * ld + h * DH;
  const bf16* obase = o + (size_t)b * Tn * D + h * DH;
  const bf16* gbase = dout + (size_t)b * Tn * D + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;
  ATTN_TR(0);

  // Prologue: EVERY global load of the staging (Q, dO, K), of delta / lse and of this wave's K / V fragments is
  // issued before the first LDS store.  Written as separate loops (the stores of one chunk before the next chunk's
  // loads) it was ~10 dependent HBM round trips per workgroup at one workgroup per CU.  nthr == 2 Tpad (one wave
  // per 32 rows), so each thread stages exactly CPR / 2 chunks of each array and delta for at most one row.
  static_assert(CPR % 2 == 0, "staging: an even number of 16-B chunks per row");
  constexpr int IT = CPR / 2;
  uint4 qv[IT], gv[IT], kv[KREG ? 1 : IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int i = tid + k * nthr, r = i / CPR, c = i - r * CPR;
    qv[k] = gv[k] = uint4{0, 0, 0, 0};
    if constexpr (!KREG) kv[k] = uint4{0, 0, 0, 0};
    if (r < Tn) {
      qv[k] = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + c * 8);
      gv[k] = *reinterpret_cast<const uint4*>(gbase + (size_t)r * D + c * 8);
      if constexpr (!KREG) kv[k] = *reinterpret_cast<const uint4*>(base + (size_t)r * ld + D + c * 8);
    }
  }
  bf16x8 orow_v[CPR], grow_v[CPR];
  float lrow = 0.0f;
  const bool drow = tid < Tn;  // delta = rowsum(dO * O) and lse of row tid (rows Tn .. Tpad - 1: 0)
  if (drow) {
#pragma unroll
    for (int c = 0; c < CPR; ++c) {
      orow_v[c] = *reinterpret_cast<const bf16x8*>(obase + (size_t)tid * D + 8 * c);
      grow_v[c] = *reinterpret_cast<const bf16x8*>(gbase + (size_t)tid * D + 8 * c);
    }
    lrow = lse[(size_t)bh * Tn + tid];
  }
  const int lane = tid & 63, wave = tid >> 6;
  const int col = lane & 31, hh = lane >> 5;
  const int kb = 32 * wave;
  const int kr = min(kb + col, Tn - 1);
  bf16x8 kf[DH / 16], vf[DH / 16];
#pragma unroll
  for (int s = 0; s < DH / 16; ++s) {
    kf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kr * ld + D + 16 * s + 8 * hh);
    vf[s] = *reinterpret_cast<const bf16x8*>(base + (size_t)kr * ld + 2 * D + 16 * s + 8 * hh);
  }
  for (int i = tid; i < DH * LDQ / 4; i += nthr) reinterpret_cast<f32x4*>(dQs)[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int i = tid + k * nthr, r = i / CPR, c = i - r * CPR;
    *reinterpret_cast<uint4*>(Qs + (size_t)r * LDR + c * 8) = qv[k];
    *reinterpret_cast<uint4*>(Gs + (size_t)r * LDR + c * 8) = gv[k];
    if constexpr (!KREG) *reinterpret_cast<uint4*>(Ks + (size_t)r * LDR + c * 8) = kv[k];
  }
  if (tid < Tpad) {
    float d = 0.0f;
    if (drow) {
#pragma unroll
      for (int c = 0; c < CPR; ++c)
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)orow_v[c][e] * (float)grow_v[c][e];
    }
    dl_s[tid] = d;
    lse_s[tid] = lrow;
  }
  __syncthreads();
  ATTN_TR(1);

  const float c2 = scale * 1.4426950408889634f;
  const bool ragged = (Tn & 31) != 0;
  f32x16 dV[NDT], dK[NDT];
#pragma unroll
  for (int t = 0; t < NDT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) dV[t][r] = dK[t][r] = 0.0f;
  const bool kmask = ragged && wave == nw - 1;  // wave-uniform: this wave holds the keys past Tn
  const bool kok = kb + col < Tn;
  bf16* dsw = dSs + (size_t)wave * 1024;
  bf16x8 kt[2];  // KREG: this wave's K rows as the dQ product's B fragments (k = key, 16 per fragment)
  if constexpr (KREG) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // 32 rows x 4 chunks of 8, two per lane
      const int i = lane + 64 * j, r = i >> 2, c = i & 3;
      uint4 x = uint4{0, 0, 0, 0};
      if (kb + r < Tn) x = *reinterpret_cast<const uint4*>(base + (size_t)(kb + r) * ld + D + c * 8);
      *reinterpret_cast<uint4*>(dsw + (size_t)r * LDR + c * 8) = x;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) kt[s2] = attn_tr_frag<LDR>(dsw, 16 * s2, 0, lane);
    // the first dS store below follows these reads in the wave's in-order LDS queue
  }

  for (int it = 0; it < nw; ++it) {
    int qt = wave + it;
    if (qt >= nw) qt -= nw;
    f32x16 S, G;
#pragma unroll
    for (int r = 0; r < 16; ++r) S[r] = G[r] = 0.0f;
#pragma unroll
    for (int s = 0; s < DH / 16; ++s) {
      const bf16x8 a = *reinterpret_cast<const bf16x8*>(Qs + (size_t)(qt * 32 + col) * LDR + 16 * s + 8 * hh);
      S = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, kf[s], S, 0, 0, 0);
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(Gs + (size_t)(qt * 32 + col) * LDR + 16 * s + 8 * hh);
      G = __builtin_amdgcn_mfma_f32_32x32x16_bf16(g, vf[s], G, 0, 0, 0);
    }
    // lse / delta of this lane's 16 queries: four runs of 4 consecutive rows (16-B LDS reads)
    const int q0 = qt * 32 + 4 * hh;
    f32x4 lq[4], dq[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lq[k] = *reinterpret_cast<const f32x4*>(lse_s + q0 + 8 * k);
      dq[k] = *reinterpret_cast<const f32x4*>(dl_s + q0 + 8 * k);
    }
    const bool qmask = ragged && qt == nw - 1;  // wave-uniform: this tile holds the queries past Tn
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float p = exp2f(S[r] * c2 - lq[r >> 2][r & 3]);
      if (kmask || qmask) p = (kok && q0 + (r & 3) + 8 * (r >> 2) < Tn) ? p : 0.0f;
      S[r] = p;
      G[r] = p * (G[r] - dq[r >> 2][r & 3]) * scale;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pa, da;
#pragma unroll
      for (int j = 0; j < 8; ++j) { pa[j] = (bf16)S[8 * s + j]; da[j] = (bf16)G[8 * s + j]; }
      const int k0 = qt * 32 + 16 * s;
#pragma unroll
      for (int t = 0; t < NDT; ++t) {
        dV[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(pa, attn_tr_frag<LDR>(Gs, k0, 32 * t, lane), dV[t], 0, 0, 0);
        dK[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(da, attn_tr_frag<LDR>(Qs, k0, 32 * t, lane), dK[t], 0, 0, 0);
      }
      // dS of this wave's keys (rows) x the tile's queries (columns) -> the wave's scratch, bf16 (the same
      // rounding the dK product above consumes)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        bf16x4 v;
        v[0] = da[4 * k]; v[1] = da[4 * k + 1]; v[2] = da[4 * k + 2]; v[3] = da[4 * k + 3];
        *reinterpret_cast<bf16x4*>(dsw + col * 32 + 16 * s + 8 * k + 4 * hh) = v;
      }
    }
    // the scratch is read back across lanes by this wave only: LDS executes a wave's operations in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // dQ[tile] += dS K: A = dS (queries on the lanes, keys k), B = K rows of this wave's keys
    f32x16 dQp[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dQp[t][r] = 0.0f;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 a = attn_tr_frag<32>(dsw, 16 * s, 0, lane);
#pragma unroll
      for (int t = 0; t < NDT; ++t)
        dQp[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
            a, KREG ? kt[s] : attn_tr_frag<LDR>(Ks, kb + 16 * s, 32 * t, lane), dQp[t], 0, 0, 0);
    }
    // lane holds dQ[q = qt*32 + (r&3) + 8(r>>2) + 4hh][d = 32t + col]: four 16-B runs of the [d][q] accumulator
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f32x4* pq = reinterpret_cast<f32x4*>(dQs + (size_t)(32 * t + col) * LDQ + q0 + 8 * k);
        f32x4 v = *pq;
        v += f32x4{dQp[t][4 * k], dQp[t][4 * k + 1], dQp[t][4 * k + 2], dQp[t][4 * k + 3]};
        *pq = v;
      }
    __syncthreads();
    ATTN_TR(2 + min(it, 11));
  }
#pragma unroll
  for (int t = 0; t < NDT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * hh;
      if (key < Tn) {
        bf16* row = dqkv + ((size_t)b * Tn + key) * ld + h * DH + 32 * t + col;
        row[D] = (bf16)dK[t][r];
        row[2 * D] = (bf16)dV[t][r];
      }
    }
  ATTN_TR(14);
  // dQ rows -> dqkv (8 head-dim values per thread, one 16-B store)
  for (int i = tid; i < Tn * CPR; i += nthr) {
    const int q = i / CPR, c = i - q * CPR;
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (bf16)dQs[(size_t)(8 * c + e) * LDQ + q];
    *reinterpret_cast<bf16x8*>(dqkv + ((size_t)b * Tn + q) * ld + h * DH + 8 * c) = v;
  }
#if TMAE_ATTN_TRACE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ATTN_TR(15);
#endif
}

// f32 (parity) form: same two phases on v_mfma_f32_32x32x2_f32, operands read straight from global memory
// (L2-resident per head); exact f32 products.
template <int DH>
__global__ void __launch_bounds__(DH == 80 ? 512 : 1024)
mha_bwd_f32_kernel(const float* __restrict__ qkv, const float* __restrict__ o, const float* __restrict__ dout,
                   const float* __restrict__ lse, float* __restrict__ dqkv, int Tn, int H, int Tpad, float scale) {
  constexpr int NDT = (DH + 31) / 32;  // columns >= DH of the last tile read as zero, never stored
  __shared__ float lse_s[1024], dl_s[1024];
  const int bh = xcd_remap(blockIdx.x, gridDim.x), b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const float* Q = qkv + (size_t)b * Tn * ld + h * DH;
  const float* K = Q + D;
  const float* V = Q + 2 * D;
  const float* Og = o + (size_t)b * Tn * D + h * DH;
  const float* G = dout + (size_t)b * Tn * D + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;
  for (int r = tid; r < Tpad; r += nthr) {
    float d = 0.0f, l = 0.0f;
    if (r < Tn) {
      for (int k = 0; k < DH; ++k) d += Og[(size_t)r * D + k] * G[(size_t)r * D + k];
      l = lse[(size_t)bh * Tn + r];
    }
    dl_s[r] = d;
    lse_s[r] = l;
  }
  __syncthreads();
  const int lane = tid & 63, wave = tid >> 6, nw = Tpad / 32;
  const int col = lane & 31, hh = lane >> 5;
  const float c2 = scale * 1.4426950408889634f;
  if (wave >= nw) return;
  auto ld_row = [&](const float* m, int row, int stride, int k) -> float {
    return row < Tn && k < DH ? m[(size_t)row * stride + k] : 0.0f;
  };
  {  // phase 1
    const int kb = 32 * wave;
    f32x16 dV[NDT], dK[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dV[t][r] = dK[t][r] = 0.0f;
    const bool kok = kb + col < Tn;
    for (int qt = 0; qt < nw; ++qt) {
      f32x16 S, P;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = P[r] = 0.0f;
      for (int kk = 0; kk < DH / 2; ++kk) {
        const int d = 2 * kk + hh;
        S = __builtin_amdgcn_mfma_f32_32x32x2f32(ld_row(Q, qt * 32 + col, ld, d), ld_row(K, kb + col, ld, d), S, 0, 0, 0);
        P = __builtin_amdgcn_mfma_f32_32x32x2f32(ld_row(G, qt * 32 + col, D, d), ld_row(V, kb + col, ld, d), P, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float p = (kok && q < Tn) ? exp2f(S[r] * c2 - lse_s[q]) : 0.0f;
        S[r] = p;
        P[r] = p * (P[r] - dl_s[q]) * scale;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
#pragma unroll
        for (int t = 0; t < NDT; ++t) {
          const int d = 32 * t + col;
          dV[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(S[r], ld_row(G, q, D, d), dV[t], 0, 0, 0);
          dK[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[r], ld_row(Q, q, ld, d), dK[t], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (key < Tn && 32 * t + col < DH) {
          float* row = dqkv + ((size_t)b * Tn + key) * ld + h * DH + 32 * t + col;
          row[D] = dK[t][r];
          row[2 * D] = dV[t][r];
        }
      }
  }
  {  // phase 2
    const int qb = 32 * wave;
    const bool qok = qb + col < Tn;
    const float lq = lse_s[qb + col], dq = dl_s[qb + col];
    f32x16 dQ[NDT];
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dQ[t][r] = 0.0f;
    for (int kt = 0; kt < nw; ++kt) {
      f32x16 S, P;
#pragma unroll
      for (int r = 0; r < 16; ++r) S[r] = P[r] = 0.0f;
      for (int kk = 0; kk < DH / 2; ++kk) {
        const int d = 2 * kk + hh;
        S = __builtin_amdgcn_mfma_f32_32x32x2f32(ld_row(K, kt * 32 + col, ld, d), ld_row(Q, qb + col, ld, d), S, 0, 0, 0);
        P = __builtin_amdgcn_mfma_f32_32x32x2f32(ld_row(V, kt * 32 + col, ld, d), ld_row(G, qb + col, D, d), P, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
        const float p = (qok && key < Tn) ? exp2f(S[r] * c2 - lq) : 0.0f;
        P[r] = p * (P[r] - dq) * scale;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * hh;
#pragma unroll
        for (int t = 0; t < NDT; ++t)
          dQ[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(P[r], ld_row(K, key, ld, 32 * t + col), dQ[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < NDT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int q = qb + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (q < Tn && 32 * t + col < DH) dqkv[((size_t)b * Tn + q) * ld + h * DH + 32 * t + col] = dQ[t][r];
      }
  }
}

// head dims on the one-pass backward (dh 80 keeps the two-phase form: its padded head-dim tile); A/B builds set
// TMAE_BWD1_DH64=0 to put the encoder's dh 64 back on the two-phase form
#ifndef TMAE_BWD1_DH64
#define TMAE_BWD1_DH64 1
#endif
template <int DH> struct AttnBwdOnePass { static constexpr bool value = DH == 32 || (DH == 64 && TMAE_BWD1_DH64); };

template <int DH>
static int mha_bwd_launch(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv, int B, int Tn,
                          int H, float scale, int dtype, hipStream_t st) {
  const int Tpad = (Tn + 31) / 32 * 32;
  const int nthr = 64 * (Tpad / 32);
  TMAE_REQUIRE(nthr <= 1024, "tmae_mha_bwd: sequence length %d too long", Tn);
  if (B * H == 0 || Tn == 0) return TMAE_OK;
  if (dtype == TMAE_BF16) {
    TMAE_REQUIRE(DH == 32 || nthr <= 512, "tmae_mha_bwd: sequence length %d too long for head dim %d", Tn, DH);
    constexpr int LDR = AttnBwd<DH>::LDR;
    // Q, dO (and K unless dh 32 holds it in registers), dS scratch, dQ, lse / delta
    const size_t lds1 = (size_t)(DH == 32 ? 2 : 3) * Tpad * LDR * 2 + (size_t)(Tpad / 32) * 2048 +
                        (size_t)DH * (Tpad + 4) * 4 + (size_t)2 * Tpad * 4;
    if (AttnBwdOnePass<DH>::value && lds1 <= 160 * 1024) {
      constexpr int D1 = AttnBwdOnePass<DH>::value ? DH : 32;
      constexpr int M9 = D1 == 32 ? 640 : 512;  // the 9-10-wave instance (dh 32 only)
      if (D1 == 32 && nthr > 512 && nthr <= 640)
        hipLaunchKernelGGL((mha_bwd1_bf16_kernel<D1, M9>), dim3(B * H), dim3(nthr), lds1, st, (const bf16*)qkv,
                           (const bf16*)o, (const bf16*)dout, lse, (bf16*)dqkv, Tn, H, Tpad, scale);
      else
        hipLaunchKernelGGL((mha_bwd1_bf16_kernel<D1>), dim3(B * H), dim3(nthr), lds1, st, (const bf16*)qkv,
                           (const bf16*)o, (const bf16*)dout, lse, (bf16*)dqkv, Tn, H, Tpad, scale);
      TMAE_LAUNCH_CHECK("tmae_mha_bwd");
    }
    const size_t lds = (size_t)2 * Tpad * LDR * 2 + (size_t)2 * Tpad * 4;
    TMAE_REQUIRE(lds <= 160 * 1024, "tmae_mha_bwd: sequence length %d needs %zu B of LDS", Tn, lds);
    hipLaunchKernelGGL((mha_bwd_bf16_kernel<DH>), dim3(B * H), dim3(nthr), lds, st, (const bf16*)qkv, (const bf16*)o,
                       (const bf16*)dout, lse, (bf16*)dqkv, Tn, H, Tpad, scale);
  } else {
    TMAE_REQUIRE(DH != 80 || nthr <= 512, "tmae_mha_bwd: sequence length %d too long for head dim 80", Tn);
    hipLaunchKernelGGL((mha_bwd_f32_kernel<DH>), dim3(B * H), dim3(nthr), 0, st, (const float*)qkv, (const float*)o,
                       (const float*)dout, lse, (float*)dqkv, Tn, H, Tpad, scale);
  }
  TMAE_LAUNCH_CHECK("tmae_mha_bwd");
}

extern "C" int tmae_mha_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv, int B,
                            int T, int H, int dh, float scale, int dtype, void* stream) {
  TMAE_REQUIRE(dh == 32 || dh == 64 || dh == 80, "tmae_mha_bwd: head dim %d unsupported (32, 64 or 80)", dh);
  TMAE_REQUIRE(qkv && o && dout && lse && dqkv, "tmae_mha_bwd: null argument");
  hipStream_t st = (hipStream_t)stream;
  if (dh == 80) return mha_bwd_launch<80>(qkv, o, dout, lse, dqkv, B, T, H, scale, dtype, st);
  return dh == 64 ? mha_bwd_launch<64>(qkv, o, dout, lse, dqkv, B, T, H, scale, dtype, st)
                  : mha_bwd_launch<32>(qkv, o, dout, lse, dqkv, B, T, H, scale, dtype, st);
}
