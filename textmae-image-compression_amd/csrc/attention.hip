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
#include "common.h"

template <typename T> struct AttnCfg;
template <> struct AttnCfg<bf16> { static constexpr int KPAD = 8, VPAD = 4, EPC = 8; };
template <> struct AttnCfg<float> { static constexpr int KPAD = 4, VPAD = 1, EPC = 4; };

template <typename T, int DH>
__global__ void __launch_bounds__(1024)
mha_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ out, int Tn, int H, int Tpad, float scale_log2e) {
  constexpr int KPAD = AttnCfg<T>::KPAD, VPAD = AttnCfg<T>::VPAD, EPC = AttnCfg<T>::EPC;
  constexpr int NDT = DH / 32;  // 32-wide output tiles along the head dim
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int ldk = DH + KPAD, ldv = Tpad + VPAD;
  T* Ks = reinterpret_cast<T*>(smem);
  T* Vt = Ks + (size_t)Tpad * ldk;

  const int bh = blockIdx.x, b = bh / H, h = bh - b * H;
  const int D = H * DH, ld = 3 * D;
  const T* base = qkv + (size_t)b * Tn * ld + h * DH;
  const int tid = threadIdx.x, nthr = blockDim.x;

  // stage K [Tpad][DH] and V^T [DH][Tpad] of this head
  constexpr int CPR = DH / EPC;  // 16-B chunks per row
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
  const float inv_l = 1.0f / l_run;
  T* orow = out + ((size_t)b * Tn + q) * D + h * DH;
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * hh;
      f32x4 v{O[dt][4 * g] * inv_l, O[dt][4 * g + 1] * inv_l, O[dt][4 * g + 2] * inv_l, O[dt][4 * g + 3] * inv_l};
      store4(orow + d, v);
    }
}

template <typename T, int DH>
static int mha_launch(const void* qkv, void* out, int B, int Tn, int H, float scale, hipStream_t st) {
  const int Tpad = (Tn + 31) / 32 * 32;
  const int nthr = 64 * (Tpad / 32);
  const size_t lds = ((size_t)Tpad * (DH + AttnCfg<T>::KPAD) + (size_t)DH * (Tpad + AttnCfg<T>::VPAD)) * sizeof(T);
  TMAE_REQUIRE(nthr <= 1024 && lds <= 160 * 1024, "tmae_mha_fwd: sequence length %d too long", Tn);
  if (B * H == 0 || Tn == 0) return TMAE_OK;
  hipLaunchKernelGGL((mha_fwd_kernel<T, DH>), dim3(B * H), dim3(nthr), lds, st, (const T*)qkv, (T*)out, Tn, H, Tpad,
                     scale * 1.4426950408889634f);
  TMAE_LAUNCH_CHECK("tmae_mha_fwd");
}

extern "C" int tmae_mha_fwd(const void* qkv, void* out, int B, int T, int H, int dh, float scale, int dtype,
                            void* stream) {
  TMAE_REQUIRE(dh == 32 || dh == 64, "tmae_mha_fwd: head dim %d unsupported (32 or 64)", dh);
  hipStream_t st = (hipStream_t)stream;
  if (dtype == TMAE_BF16) return dh == 64 ? mha_launch<bf16, 64>(qkv, out, B, T, H, scale, st)
                                          : mha_launch<bf16, 32>(qkv, out, B, T, H, scale, st);
  return dh == 64 ? mha_launch<float, 64>(qkv, out, B, T, H, scale, st)
                  : mha_launch<float, 32>(qkv, out, B, T, H, scale, st);
}
