// Shared definitions for the gfx950 (CDNA4 / MI355X) kernels behind libtmae.so.
//
// Everything here is written for one target: 64-lane wavefronts, MFMA matrix cores,
// 160 KiB LDS per CU.  No CUDA dialect, no dual-platform macros.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/tmae.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// ---------------------------------------------------------------- host-side error plumbing
void tmae_set_error(int code, const char* fmt, ...);

#define TMAE_REQUIRE(cond, ...)                           \
  do {                                                    \
    if (!(cond)) {                                        \
      tmae_set_error(TMAE_EINVAL, __VA_ARGS__);           \
      return TMAE_EINVAL;                                 \
    }                                                     \
  } while (0)

#define TMAE_LAUNCH_CHECK(name)                                              \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) {                                                  \
      tmae_set_error(TMAE_EHIP, "%s: launch failed: %s", name,               \
                     hipGetErrorString(_e));                                 \
      return TMAE_EHIP;                                                      \
    }                                                                        \
    return TMAE_OK;                                                          \
  } while (0)

// the same check between two launches of one entry point (returns only on failure)
#define TMAE_LAUNCH_CHECK_NORET(name)                                        \
  do {                                                                       \
    hipError_t _e = hipGetLastError();                                       \
    if (_e != hipSuccess) {                                                  \
      tmae_set_error(TMAE_EHIP, "%s: launch failed: %s", name,               \
                     hipGetErrorString(_e));                                 \
      return TMAE_EHIP;                                                      \
    }                                                                        \
  } while (0)

// ---------------------------------------------------------------- device helpers
__device__ __forceinline__ float gelu_erf(float x) {
  // nn.GELU() default (approximate='none'): 0.5 * x * (1 + erf(x / sqrt(2))).
  // libm erff expands to ~70 VALU ops per element, which made the fc1 / conv epilogues the
  // kernels' critical path (PMC: 10x more VALU than MFMA instructions).  Abramowitz-Stegun 7.1.26
  // costs one v_rcp, one v_exp and six FMAs; |erf error| <= 1.5e-7 (4.4e-7 measured in f32), so
  // |GELU error| <= 3.5e-7 absolute -- below f32 rounding of O(1) activations.
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);  // exp(-z^2)
  const float erf_abs = fmaf(-p, e, 1.0f);
  // 0.5 x (1 + sign(x) erf|z|): for x >= 0 -> 0.5 x (1 + erf_abs); for x < 0 -> 0.5 x (1 - erf_abs) = 0.5 x p e
  const float h = 0.5f * x;
  return x >= 0.0f ? fmaf(h, erf_abs, h) : h * p * e;
}

// GELU for bf16 outputs: x * sigmoid(x (a + b x^2 + c x^4)), coefficients fitted to the erf GELU by
// minimax over [-10, 10] (x clamped there inside the sigmoid, saturated beyond): |error| <= 2.6e-5 absolute, far below bf16 resolution of the stored value
// (half an ulp is 2^-9 relative).  One v_exp + one v_rcp + five FMA-class ops against gelu_erf's
// fifteen: the GELU of the fc1 / decoder-fc1 epilogues was 14 us of a 74 us launch.  The log2(e)
// of exp is folded into the coefficients.  Large |x|: exp2 -> inf gives 0 (x < 0), exp2 -> 0 gives x.
__device__ __forceinline__ float gelu_bf16out(float x) {
  const float xc = __builtin_amdgcn_fmed3f(x, -10.0f, 10.0f);  // the quintic turns over past |x| ~ 11
  const float x2 = xc * xc;
  const float z = xc * fmaf(fmaf(1.0142631e-3f, x2, -0.10677572f), x2, -2.3011213f);  // -log2e (a + b x2 + c x4)
  return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(z));
}
// the same on two values with packed f32 math (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32: two lanes' worth of
// FMA-class work per issue; bitwise equal to gelu_bf16out, same operations in the same order)
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu2_bf16out(f32x2 x) {
  const f32x2 xc = {__builtin_amdgcn_fmed3f(x.x, -10.0f, 10.0f), __builtin_amdgcn_fmed3f(x.y, -10.0f, 10.0f)};
  const f32x2 x2 = xc * xc;
  f32x2 p = __builtin_elementwise_fma((f32x2){1.0142631e-3f, 1.0142631e-3f}, x2, (f32x2){-0.10677572f, -0.10677572f});
  p = __builtin_elementwise_fma(p, x2, (f32x2){-2.3011213f, -2.3011213f});
  const f32x2 z = xc * p;
  const f32x2 d = (f32x2){1.0f, 1.0f} + (f32x2){__builtin_amdgcn_exp2f(z.x), __builtin_amdgcn_exp2f(z.y)};
  return x * (f32x2){__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ void gelu8_bf16out(f32x4& lo, f32x4& hi) {
  lo.xy = gelu2_bf16out(lo.xy);
  lo.zw = gelu2_bf16out(lo.zw);
  hi.xy = gelu2_bf16out(hi.xy);
  hi.zw = gelu2_bf16out(hi.zw);
}
// GELU derivative (training data gradients: the GEMM epilogues in train.hip, the fused stack backward)
__device__ __forceinline__ float gelu_grad(float x) {
  // d/dx [0.5 x (1 + erf(x / sqrt2))] = Phi(x) + x phi(x); erf by Abramowitz-Stegun 7.1.26 like gelu_erf
  const float z = fabsf(x) * 0.70710678118654752440f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  p *= t;
  const float e = __builtin_amdgcn_exp2f(-z * z * 1.44269504088896341f);  // exp(-x^2 / 2)
  const float erf_abs = fmaf(-p, e, 1.0f);
  const float cdf = x >= 0.0f ? 0.5f + 0.5f * erf_abs : 0.5f * p * e;
  return cdf + x * e * 0.39894228040143267794f;
}

// gelu_grad on two values with packed f32 math (v_pk_fma / v_pk_mul): the same approximation as the scalar
// form, ~12 VALU issues per element instead of ~19; the data-gradient epilogues apply it to every fc1 / conv
// element
__device__ __forceinline__ f32x2 gelu_grad2(f32x2 x) {
  const f32x2 z = (f32x2){fabsf(x.x), fabsf(x.y)} * 0.70710678118654752440f;
  const f32x2 d = __builtin_elementwise_fma((f32x2){0.3275911f, 0.3275911f}, z, (f32x2){1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  f32x2 p = __builtin_elementwise_fma((f32x2){1.061405429f, 1.061405429f}, t, (f32x2){-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, (f32x2){1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, (f32x2){-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, (f32x2){0.254829592f, 0.254829592f});
  p *= t;
  const f32x2 a = -z * z * 1.44269504088896341f;
  const f32x2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  const f32x2 erf_abs = __builtin_elementwise_fma(-p, e, (f32x2){1.0f, 1.0f});
  const f32x2 pos = 0.5f + 0.5f * erf_abs, neg = 0.5f * p * e;
  const f32x2 cdf = {x.x >= 0.0f ? pos.x : neg.x, x.y >= 0.0f ? pos.y : neg.y};
  return cdf + x * e * 0.39894228040143267794f;
}

// the GELU an epilogue storing OT applies
template <typename OT> __device__ __forceinline__ float gelu_for(float x) {
  if constexpr (sizeof(OT) == 2) return gelu_bf16out(x);
  else return gelu_erf(x);
}

template <typename T> __device__ __forceinline__ T to_out(float v);
template <> __device__ __forceinline__ float to_out<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16 to_out<bf16>(float v) { return (bf16)v; }

__device__ __forceinline__ float bf_to_f(bf16 v) { return (float)v; }

// store 4 consecutive values (16 B for f32, 8 B for bf16)
__device__ __forceinline__ void store4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
__device__ __forceinline__ void store4(bf16* p, f32x4 v) {
  bf16x4 o;
  o[0] = (bf16)v[0]; o[1] = (bf16)v[1]; o[2] = (bf16)v[2]; o[3] = (bf16)v[3];
  *reinterpret_cast<bf16x4*>(p) = o;
}
__device__ __forceinline__ f32x4 load4f(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ f32x4 load4f(const bf16* p) {
  bf16x4 v = *reinterpret_cast<const bf16x4*>(p);
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}

// 8 consecutive values: one 16-B store for bf16, two for f32
__device__ __forceinline__ void store8(float* p, f32x4 lo, f32x4 hi) {
  *reinterpret_cast<f32x4*>(p) = lo;
  *reinterpret_cast<f32x4*>(p + 4) = hi;
}
__device__ __forceinline__ void store8(bf16* p, f32x4 lo, f32x4 hi) {
  bf16x8 o;
  o[0] = (bf16)lo[0]; o[1] = (bf16)lo[1]; o[2] = (bf16)lo[2]; o[3] = (bf16)lo[3];
  o[4] = (bf16)hi[0]; o[5] = (bf16)hi[1]; o[6] = (bf16)hi[2]; o[7] = (bf16)hi[3];
  *reinterpret_cast<bf16x8*>(p) = o;
}
__device__ __forceinline__ void load8f(const float* p, f32x4& lo, f32x4& hi) {
  lo = *reinterpret_cast<const f32x4*>(p);
  hi = *reinterpret_cast<const f32x4*>(p + 4);
}
__device__ __forceinline__ void load8f(const bf16* p, f32x4& lo, f32x4& hi) {
  const bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
  lo = f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
  hi = f32x4{(float)v[4], (float)v[5], (float)v[6], (float)v[7]};
}

// 16-byte chunk of 8 bf16 from 8 floats (two 16-B loads)
__device__ __forceinline__ uint4 pack8_bf16(f32x4 a, f32x4 b) {
  bf16x8 o;
  o[0] = (bf16)a[0]; o[1] = (bf16)a[1]; o[2] = (bf16)a[2]; o[3] = (bf16)a[3];
  o[4] = (bf16)b[0]; o[5] = (bf16)b[1]; o[6] = (bf16)b[2]; o[7] = (bf16)b[3];
  return *reinterpret_cast<uint4*>(&o);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks b and b+8 land on one XCD; give each XCD a contiguous run of logical tiles.
// Sum over the 64 lanes of a wave, every lane getting the total, without the LDS crossbar: DPP quad permutes
// (xor 1, xor 2) and row mirrors (8, 16 lanes) leave each 16-lane row's sum in all its lanes, then the four row
// sums are read lane-uniformly (v_readlane) and added as (r0 + r1) + (r2 + r3).  Every lane ends with the same
// bits.  (A __shfl_xor butterfly is six ds_bpermute round trips through the LDS unit.)  Whole wave active.
#define TMAE_DPP_ADD(v, ctrl)                                                                                      \
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), ctrl, 0xF, 0xF, true))
__device__ __forceinline__ float wave_allsum(float v) {
  TMAE_DPP_ADD(v, 0xB1);   // quad_perm [1,0,3,2]: xor 1
  TMAE_DPP_ADD(v, 0x4E);   // quad_perm [2,3,0,1]: xor 2
  TMAE_DPP_ADD(v, 0x141);  // row_half_mirror: the other quad of each 8
  TMAE_DPP_ADD(v, 0x140);  // row_mirror: the other 8 of each 16
  const int b = __builtin_bit_cast(int, v);
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48));
  return (r0 + r1) + (r2 + r3);
}
#undef TMAE_DPP_ADD

__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

static inline int ceil_div(int a, int b) { return (a + b - 1) / b; }
