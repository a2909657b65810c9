// One whole slice-transform stack per workgroup, activations resident in LDS (bf16).
//
// cc_transform_mean[i] / cc_transform_scale[i] / lrp_transform[i] (MCM.py:165-293, applied at
// MCM.py:761-784) are five 3x3 convs (224 -> 176 -> 128 -> 80 -> 32 channels at the default config)
// with GELU between them, over the 12x12 latent grid.  Run layer by layer (conv_halo.h) every layer is
// a separate launch of 64-256 workgroups whose ~0.7 us per (chunk, tap) step chain, not the MFMA rate,
// sets the time, and the serial slice chain (slices 0..5) is a row of such launches.  Here ONE
// workgroup owns one (problem, image) and runs the whole stack:
//   * the layer-0 input (y_hat slices, MCM.py:756-760, torch.cat of two sources without a copy) goes
//     global -> LDS once; every layer's output stays in LDS (two ping-pong buffers, 144 rows of up to
//     224 channels each) and is the next layer's input -- no HBM round trip between layers;
//   * weights never touch LDS: they are pre-packed in MFMA fragment order ([tap][k32][cout16][lane][8])
//     so every A-fragment is one coalesced 1-KiB wave load from L2 (all images of a problem share them),
//     prefetched 4-6 K-steps ahead into VGPRs; so the K loop has NO workgroup barrier at all, only the
//     one between layers;
//   * pixel fragments are 16 consecutive pixels; tap (dy, dx) shifts the LDS row by dy*G + dx, pixels
//     whose tap falls outside the grid read the matching row of a 16-row zero block.  Row pitch =
//     2 * round32(C) + 32 bytes, so every fragment read is bank-conflict-free for every tap shift.
// Work split: 8 waves (two per SIMD); a wave item = two 16-channel output fragments x all 9 pixel
// fragments (224-wide layers), x a pixel half (176 / 128), or one fragment x a half (80 / 32); items
// dealt round-robin to the waves (the layer loop below).
// Chain mode (TMAE_LIC_STACK_CHAIN): a slice's mean-stack workgroups go on with the slice's lrp stack.
// MFMA v_mfma_f32_16x16x32_bf16 issued swapped (A = weights 16 couts x 32 k, B = 32 k x 16 pixels):
// each lane ends with 4 consecutive output channels of one pixel (one 8-B LDS store per fragment).
// The first layer's epilogue adds the latent-channel partial sums (the P buffer of mcm.py _slices) and
// the last layer's writes mu / sigma (f32) or, for lrp, y_hat = y_hat_pre + 0.5 tanh(.) (MCM.py:779-784).
#include "gemm_core.h"

namespace lstk {
constexpr int NW = 8;                       // waves per workgroup (two per SIMD: 256 VGPRs each)
constexpr int MAXC = 224;                   // widest resident activation (channels, padded to 32)
constexpr int MAXPITCH = 2 * MAXC + 32;     // bytes
constexpr int MAXPIX = 144;                 // 12 x 12
constexpr int BUF = MAXPIX * MAXPITCH;      // one activation buffer
constexpr int ZOFF = 2 * BUF;               // zero block: 16 rows, read by taps that fall outside the grid
constexpr int TMASK = 2 * BUF + 16 * MAXPITCH;  // per-pixel 9-bit tap-validity masks (u16, 160 pixel slots)
constexpr int LDS_BYTES = TMASK + 320;
__host__ __device__ constexpr int pad32(int c) { return (c + 31) & ~31; }
// row pitch: 32 B past the channels makes every ds_read_b128 fragment read (16 consecutive rows, the
// gfx950 lane groups {0-3,12-15,20-27} / {4-11,16-19,28-31} mixing two k-chunks) conflict-free for every
// tap shift; 16 B left them 2-way conflicted
__host__ __device__ constexpr int pitch(int c) { return 2 * pad32(c) + 32; }
}  // namespace lstk

struct LstkLayer {
  const bf16* w;
  const float* b;
  int cin, cout;
};

// the argument block is read in place from the kernarg segment (scalar loads, layer fields indexed at
// run time): a by-value copy indexed by the layer number would live in scratch
typedef const __attribute__((address_space(4))) tmae_lic_stack_args LstkArgs;

// per-workgroup outputs of the last layer / the layer-0 addend, problem offsets applied
struct LstkOut {
  const float* add;
  int ld_add;
  void* y;
  int ldy, y_f32;
  const float* src;
  int ld_src;
  void* y2;
  int ldy2;
  bf16* sp;   // training: this layer's pre-activation, bf16 [rows][cout] (NULL: not kept)
  bf16* sa;   // training: its GELU output
  float* st;  // training, lrp last layer: the pre-tanh value, f32 [rows][cout]
  int bwd;    // TMAE_LIC_STACK_BWD: out = acc * GELU'(sp) -> sa (global) and, but for the last layer, LDS
  int route;  // TMAE_LIC_STACK_BWD, last layer with racc: f32 += into the channel-range accumulators,
  LstkArgs* ra;  // read from the kernarg block at the epilogue (copies held per layer spilled SGPRs to scratch)
  int rb1;       // the problem index the route strides apply to
  int trl;       // LSTK_TRACE: the layer's trace slot base
};

#ifndef LSTK_OPT
#define LSTK_OPT 0  // A/B builds: 1 = 8-B GELU epilogue stores (no permlane16_swap pairing)
#endif
#ifndef LSTK_DIAG
#define LSTK_DIAG 0  // phase isolation builds (tools/lstk_diag.sh): 4 = no MFMA, 8 = no B reads, 16 = no A loads,
                     // 32 = no epilogue, 64 = no layer-0 addend loads, 128 = no GELU (bias only)
#endif

#ifndef LSTK_TRACE
#define LSTK_TRACE 0  // timeline builds (tools/lstk_trace.py): per wave and layer, K-loop / epilogue cycles, done / exit times
#endif
#if LSTK_TRACE
// [workgroup][wave][48] shader-clock stamps (s_memtime): 0 start, 1 after the prologue barrier, then per layer slot
// 2 + 4 l: layer start, K-loop cycles, epilogue cycles, items done; 47 end.  One writer per slot (lane 0).
constexpr int LSTK_TR_WG = 1024, LSTK_TR_SLOTS = 48;
__device__ unsigned long long g_lstk_trace[LSTK_TR_WG * 8 * LSTK_TR_SLOTS];
__device__ __forceinline__ unsigned long long* lstk_tr_slot(int s) {
  const int wg = blockIdx.x < LSTK_TR_WG ? blockIdx.x : LSTK_TR_WG - 1;
  return g_lstk_trace + ((size_t)wg * 8 + (threadIdx.x >> 6)) * LSTK_TR_SLOTS + s;
}
__device__ __forceinline__ void lstk_tr_set(int s, unsigned long long v) {
  if ((threadIdx.x & 63) == 0) *lstk_tr_slot(s) = v;
}
__device__ __forceinline__ void lstk_tr_add(int s, unsigned long long v) {
  if ((threadIdx.x & 63) == 0) *lstk_tr_slot(s) += v;
}
extern "C" int tmae_lstk_trace_read(void* dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_lstk_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" int tmae_lstk_trace_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_lstk_trace)) != hipSuccess) return 1;
  return hipMemset(p, 0, sizeof(g_lstk_trace)) == hipSuccess ? 0 : 1;
}
#endif

__device__ __forceinline__ bf16x8 lstk_lds8(const unsigned char* lb, unsigned off) {
#if LSTK_DIAG & 8
  bf16x8 v;
  asm volatile("; no B read %0" : "=v"(v) : "v"(off));
  return v;
#else
  return *reinterpret_cast<const bf16x8*>(lb + off);
#endif
}

// One wave item: NF output fragments (channels 16 f0 .. 16 (f0 + NF) - 1) x MF pixel fragments
// j0 .. j0 + MF - 1, NKC = K-steps of 32 input channels per tap.  Every B fragment read from LDS feeds NF
// MFMAs (at NF = 1 one 1-KiB read per 16-cycle MFMA on each SIMD is exactly the LDS array's 256 B/clk).
// All 9 x NKC K-steps are unrolled: A fragments stream through a static register ring D steps ahead,
// B fragments are read one step ahead.
template <int NF, int MF, int NKC, bool BWD>
__device__ __forceinline__ void lstk_item(const LstkLayer& L, bool first, bool last, const LstkOut& o, int img,
                                          int f0, int j0, unsigned char* lb, unsigned in_off, unsigned out_off,
                                          int npix, int G, int lane) {
  using namespace lstk;
  // opaque per item: keeps the per-fragment pixel / address math inside the item (hoisted out of the
  // layer loop it was ~70 VGPRs of 64-bit epilogue addresses, all spilled)
  asm volatile("" : "+v"(lane));
#if LSTK_TRACE
  const unsigned long long tr_a = __builtin_amdgcn_s_memtime();
#endif
  const int fr = lane & 15, fq = lane >> 4;
  const int nfr = (L.cout + 15) >> 4;
  f32x4 acc[NF][MF];
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (NKC > 0) {
    const int pin = pitch(L.cin);
    // A fragment of step s = tap * NKC + kc, output fragment f at w + ((s * nfr + f) * 64 + lane) * 8;
    // fragments past nfr (odd nfr at NF = 2) re-read fragment nfr - 1 and are dropped in the epilogue
    const bf16* wp[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) wp[i] = L.w + ((size_t)min(f0 + i, nfr - 1) * 64 + lane) * 8;
    const unsigned sstride = (unsigned)nfr * 512u;
    // A ring: step s's fragments in slot s % D, the load of step s + D issued right after slot s is read;
    // all 9 x NKC steps are unrolled so the slots are static registers (a rolled tap loop needed copies
    // of the in-flight loads at its back edge, i.e. a vmcnt(0) at the end of every tap)
    constexpr int NS = 9 * NKC, D = NF == 2 ? 4 : 6;
    bf16x8 ar[D][NF];
    const bf16* wl[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      wl[i] = wp[i];
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (d < NS) {
          ar[d][i] = *reinterpret_cast<const bf16x8*>(wl[i]);
          wl[i] += sstride;
        }
    }
    // per pixel fragment: bit t set when tap t of this lane's pixel lies inside the grid (table built once
    // per workgroup in LDS; 0 for pixels past the grid)
    unsigned tmask[MF];
#pragma unroll
    for (int j = 0; j < MF; ++j) tmask[j] = *reinterpret_cast<const unsigned short*>(lb + TMASK + 2 * (16 * (j0 + j) + fr));
    auto row = [&](int t, int j) -> unsigned {
      const int p = 16 * (j0 + j) + fr, sh = (t / 3 - 1) * G + (t % 3 - 1);
      // an outside tap reads zero row (p + sh) mod 16 of the zero block: the same bank quad as an inside
      // row would give, so border fragments stay conflict-free
      const unsigned r = (unsigned)(p + sh);
      return ((tmask[j] >> t) & 1u ? in_off + r * pin : (unsigned)ZOFF + (r & 15u) * pin) + 16u * fq;
    };
    // B fragments double-buffered: step s+1's reads are issued before step s's MFMAs; the sched barrier
    // keeps the scheduler from hoisting later steps' reads
    bf16x8 bv[2][MF];
#pragma unroll
    for (int j = 0; j < MF; ++j) bv[0][j] = lstk_lds8(lb, row(0, j));
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (s + 1 < NS) {
        const int t1 = (s + 1) / NKC, k1 = (s + 1) - t1 * NKC;
#pragma unroll
        for (int j = 0; j < MF; ++j) bv[(s + 1) & 1][j] = lstk_lds8(lb, row(t1, j) + 64u * k1);
      }
      bf16x8 a0[NF];
#pragma unroll
      for (int i = 0; i < NF; ++i) {
        a0[i] = ar[s % D][i];
        if (s + D < NS && !(LSTK_DIAG & 16)) {
          ar[s % D][i] = *reinterpret_cast<const bf16x8*>(wl[i]);
          wl[i] += sstride;  // one pointer bump per load (per-step constant offsets spilled ~280 SGPRs)
        }
      }
#if LSTK_DIAG & 4  // phase isolation: no MFMA (operands consumed by an empty asm)
#pragma unroll
      for (int j = 0; j < MF; ++j) asm volatile("" ::"v"(bv[s & 1][j]));
#pragma unroll
      for (int i = 0; i < NF; ++i) asm volatile("" ::"v"(a0[i]));
#else
#pragma unroll
      for (int j = 0; j < MF; ++j)
#pragma unroll
        for (int i = 0; i < NF; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], bv[s & 1][j], acc[i][j], 0, 0, 0);
#endif
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // (Round 6 measured the bias loaded before the K loop -- ms_3 65.3-65.9 vs 65.7-66.1 us, profiles/r06/c4_lstk.txt
  // -- and a deferred epilogue: a wave's two items of a hidden layer, the first item's GELU / LDS stores issued inside
  // the second item's K loop, bitwise the same outputs, ms_3 65.5 vs 65.3 us and the forward 9806 / 9823 vs
  // 9862 / 9855 img/s same box, c7_*: the K loops do not leave the MFMA pipe idle enough for the epilogue's VALU to
  // hide in.  Neither was kept.)
  // epilogue: lane holds channels c..c+3 of pixel 16 (j0 + j) + fr
#if LSTK_TRACE
  const unsigned long long tr_b = __builtin_amdgcn_s_memtime();
  lstk_tr_add(o.trl + 1, tr_b - tr_a);
  struct TrEnd {
    unsigned long long b;
    int slot;
    __device__ ~TrEnd() { lstk_tr_add(slot, __builtin_amdgcn_s_memtime() - b); }
  } tr_end{tr_b, o.trl + 2};
#endif
#if LSTK_DIAG & 32  // phase isolation: no epilogue (keep the accumulators alive)
#pragma unroll
  for (int i = 0; i < NF; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) asm volatile("" ::"v"(acc[i][j]));
  return;
#endif
  // Every global operand of the epilogue (the layer-0 addend, the lrp source) is loaded for all
  // fragments first, then the math runs: fetched per fragment, each load was its own exposed round trip
  // (vmcnt(0) per fragment).  Lanes past cout / npix use a clamped address and drop their result.
  const int pout = pitch(L.cout);
  int cc[NF];
  bool okc[NF];
  f32x4 bias[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    cc[i] = 16 * (f0 + i) + 4 * fq;
    okc[i] = cc[i] < L.cout;
    bias[i] = BWD ? f32x4{0.f, 0.f, 0.f, 0.f} : load4f(L.b + (okc[i] ? cc[i] : 0));
  }
  auto pix = [&](int j) { return 16 * (j0 + j) + fr; };
  auto grow = [&](int j) { return (size_t)img * npix + (size_t)min(pix(j), npix - 1); };
  if constexpr (BWD) {
  if (o.route) {
    // the stack's first conv's input gradient, routed by channel range into f32 accumulators (+=); the 4
    // channels of a lane never straddle a range (limits are multiples of 4)
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      if (!okc[i]) continue;
      const int c = cc[i];
      const int l0 = o.ra->rlim[0], l1 = o.ra->rlim[1];
      const int r = c < l0 ? 0 : (c < l1 ? 1 : 2);
      const int c0 = r == 0 ? 0 : (r == 1 ? l0 : l1);
      const int ld = o.ra->rld[r];
      float* base = o.ra->racc[r] + o.rb1 * o.ra->rs[r] + (c - c0);
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        if (pix(j) >= npix) continue;
        float* q = base + grow(j) * ld;
        store4(q, load4f(q) + acc[i][j]);
      }
    }
    return;
  }
  {
    // data gradient: the forward's GELU inputs of these channels, loaded for the whole item first
    f32x4 pv[NF][MF];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) pv[i][j] = load4f(o.sp + grow(j) * L.cout + (okc[i] ? cc[i] : 0));
    const int pout = pitch(L.cout);
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const f32x2 g0 = gelu_grad2(pv[i][j].xy), g1 = gelu_grad2(pv[i][j].zw);
        f32x4 v = acc[i][j];
        v[0] *= g0.x; v[1] *= g0.y; v[2] *= g1.x; v[3] *= g1.y;
        bf16x4 q;
        q[0] = (bf16)v[0]; q[1] = (bf16)v[1]; q[2] = (bf16)v[2]; q[3] = (bf16)v[3];
        if (okc[i] && pix(j) < npix) {
          *reinterpret_cast<bf16x4*>(o.sa + grow(j) * L.cout + cc[i]) = q;
          if (!last) *reinterpret_cast<bf16x4*>(lb + out_off + pix(j) * pout + 2 * cc[i]) = q;
        }
      }
    return;
  }
  } else {  // forward
  if (!last) {
    if (first && o.add && !(LSTK_DIAG & 64)) {
      f32x4 ad[NF][MF];
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) ad[i][j] = load4f(o.add + grow(j) * o.ld_add + (okc[i] ? cc[i] : 0));
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) acc[i][j] += ad[i][j];
    }
    auto gelu4 = [&](int i, int j) {
      const f32x4 v = acc[i][j] + bias[i];
#if LSTK_DIAG & 128
      const f32x2 lo = v.xy, hi = v.zw;
#else
      const f32x2 lo = gelu2_bf16out(v.xy), hi = gelu2_bf16out(v.zw);
#endif
      bf16x4 q;
      q[0] = (bf16)lo.x; q[1] = (bf16)lo.y; q[2] = (bf16)hi.x; q[3] = (bf16)hi.y;
      if (o.sp && okc[i] && pix(j) < npix) {  // training: keep the GELU input and output for the backward
        store4(o.sp + grow(j) * L.cout + cc[i], v);
        *reinterpret_cast<bf16x4*>(o.sa + grow(j) * L.cout + cc[i]) = q;
      }
      return q;
    };
    if (NF == 2 && (L.cout & 7) == 0 && !(LSTK_OPT & 1)) {
      // v_permlane16_swap pairs lane rows (fq, fq ^ 1): even rows gather 8 consecutive channels of
      // fragment 0, odd rows of fragment 1, so each lane stores 16 B per pixel fragment (one ds_write_b128
      // instead of two ds_write_b64 with 4-way bank conflicts)
      const int ch = 16 * (f0 + (fq & 1)) + 4 * (fq & 2);
      const bool okw = ch < L.cout;
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const bf16x4 qa = gelu4(0, j), qb = gelu4(NF - 1, j);
        const uint2 ua = *reinterpret_cast<const uint2*>(&qa), ub = *reinterpret_cast<const uint2*>(&qb);
        const auto r0 = __builtin_amdgcn_permlane16_swap(ua.x, ub.x, false, false);
        const auto r1 = __builtin_amdgcn_permlane16_swap(ua.y, ub.y, false, false);
        if (okw && pix(j) < npix)
          *reinterpret_cast<uint4*>(lb + out_off + pix(j) * pout + 2 * ch) = uint4{r0[0], r1[0], r0[1], r1[1]};
      }
    } else {
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < MF; ++j) {
          const bf16x4 q = gelu4(i, j);
          if (okc[i] && pix(j) < npix) *reinterpret_cast<bf16x4*>(lb + out_off + pix(j) * pout + 2 * cc[i]) = q;
        }
    }
  } else if (o.src) {  // lrp: y_hat = y_hat_pre + 0.5 tanh(lrp)
    f32x4 sv[NF][MF];
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) sv[i][j] = load4f(o.src + grow(j) * o.ld_src + (okc[i] ? cc[i] : 0));
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const f32x4 v = acc[i][j] + bias[i];
        f32x4 r = sv[i][j];
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] += 0.5f * tanhf(v[e]);
        if (okc[i] && pix(j) < npix) {
          if (o.st) store4(o.st + grow(j) * L.cout + cc[i], v);
          store4(reinterpret_cast<bf16*>(o.y) + grow(j) * o.ldy + cc[i], r);
          if (o.y2) store4(reinterpret_cast<bf16*>(o.y2) + grow(j) * o.ldy2 + cc[i], r);
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < NF; ++i)
#pragma unroll
      for (int j = 0; j < MF; ++j) {
        const f32x4 v = acc[i][j] + bias[i];
        if (okc[i] && pix(j) < npix) {
          if (o.y_f32) store4(reinterpret_cast<float*>(o.y) + grow(j) * o.ldy + cc[i], v);
          else store4(reinterpret_cast<bf16*>(o.y) + grow(j) * o.ldy + cc[i], v);
        }
      }
  }
  }  // forward
}

template <int NF, int MF, bool BWD>
__device__ __forceinline__ void lstk_dispatch(int nkc, const LstkLayer& L, bool first, bool last, const LstkOut& o,
                                              int img, int f0, int j0, unsigned char* lb, unsigned in_off,
                                              unsigned out_off, int npix, int G, int lane) {
#define LSTK_CASE(K) \
  case K: lstk_item<NF, MF, K, BWD>(L, first, last, o, img, f0, j0, lb, in_off, out_off, npix, G, lane); break;
  switch (nkc) {
    LSTK_CASE(0) LSTK_CASE(1) LSTK_CASE(2) LSTK_CASE(3) LSTK_CASE(4) LSTK_CASE(5) LSTK_CASE(6) LSTK_CASE(7)
    default: break;
  }
#undef LSTK_CASE
}


// BWD (TMAE_LIC_STACK_BWD) is its own instantiation: the backward epilogue's registers stay out of the forward's
template <bool BWD>
__global__ void __launch_bounds__(lstk::NW * 64) lic_stack_kernel(tmae_lic_stack_args) {
  using namespace lstk;
  LstkArgs* a = (LstkArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  __shared__ __attribute__((aligned(16))) uint4 lds[LDS_BYTES / 16];
  unsigned char* lb = reinterpret_cast<unsigned char*>(lds);
  const int n = a->n, G = a->G, npix = G * G, nmf = (npix + 15) >> 4, nb2 = a->nb2;
  const int t = xcd_remap(blockIdx.x, gridDim.x);  // each XCD's L2 serves a contiguous run of problems
  const int prob = t / n, img = t - prob * n;
  // chained launches interleave mean (two stacks) and scale (one stack) problems, so every XCD's run of
  // logical workgroups carries the same mix of long and short ones
  const bool ilv = a->flags & TMAE_LIC_STACK_CHAIN;
  const long long b1 = ilv ? prob % a->nb1 : prob / nb2, b2 = ilv ? prob / a->nb1 : prob - (prob / nb2) * nb2;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#if LSTK_TRACE
  lstk_tr_set(0, __builtin_amdgcn_s_memtime());
#endif

  // zero row + layer-0 input -> buffer 0 (channels [0, c1) from x1, [c1, cin0) from x2, pad zeros)
  for (int i = tid; i < 16 * MAXPITCH / 16; i += NW * 64) reinterpret_cast<uint4*>(lds)[ZOFF / 16 + i] = uint4{0, 0, 0, 0};
  for (int p = tid; p < 160; p += NW * 64) {
    unsigned m = 0;
    if (p < npix) {
      const int py = p / G, px = p - py * G;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = py + t / 3 - 1, xx = px + t % 3 - 1;
        m |= ((unsigned)yy < (unsigned)G && (unsigned)xx < (unsigned)G) ? (1u << t) : 0u;
      }
    }
    *reinterpret_cast<unsigned short*>(lb + TMASK + 2 * p) = (unsigned short)m;
  }
  const int c1 = a->c1, cin0 = a->c1 + a->c2;
  const int nl = a->nlayers;
  {
    const bf16* x1 = reinterpret_cast<const bf16*>(a->x1) + b1 * a->x1_s[0] + b2 * a->x1_s[1];
    const bf16* x2 = a->x2 ? reinterpret_cast<const bf16*>(a->x2) + b1 * a->x2_s[0] + b2 * a->x2_s[1] : nullptr;
    const int ld1 = a->ld1, ld2 = a->ld2;
    const int q = pad32(cin0) >> 3, pin = pitch(cin0);
    for (int i = tid; i < npix * q; i += NW * 64) {
      const int p = i / q, ch = 8 * (i - p * q);
      const size_t row = (size_t)img * npix + p;
      uint4 v = uint4{0, 0, 0, 0};
      if (ch < c1) v = *reinterpret_cast<const uint4*>(x1 + row * ld1 + ch);
      else if (ch < cin0) v = *reinterpret_cast<const uint4*>(x2 + row * ld2 + (ch - c1));
      *reinterpret_cast<uint4*>(lb + p * pin + 2 * ch) = v;
    }
  }
  __syncthreads();
#if LSTK_TRACE
  lstk_tr_set(1, __builtin_amdgcn_s_memtime());
  int tr_layer = 0;
#endif

  // pass 0: the stack of this problem; pass 1 (TMAE_LIC_STACK_CHAIN, problem (0, 0) = a slice's mean stack):
  // that slice's lrp stack, same workgroup, its input built from the mean stack's output
  const bool chain = (a->flags & TMAE_LIC_STACK_CHAIN) && b1 == 0;
  int cin = cin0;
  for (int pass = 0; pass < (chain ? 2 : 1); ++pass) {
    LstkOut o;
    o.bwd = BWD;
    o.route = 0;
    if (pass == 0) {
      o.add = a->addend ? a->addend + b1 * a->a_s[0] + b2 * a->a_s[1] : nullptr;
      o.ld_add = a->ld_add;
      o.y_f32 = a->y_f32;
      o.y = !a->y ? nullptr
            : o.y_f32 ? (void*)(reinterpret_cast<float*>(a->y) + b1 * a->y_s[0] + b2 * a->y_s[1])
                      : (void*)(reinterpret_cast<bf16*>(a->y) + b1 * a->y_s[0] + b2 * a->y_s[1]);
      o.ldy = a->ldy;
      o.src = a->lrp_src ? a->lrp_src + b1 * a->src_s[0] + b2 * a->src_s[1] : nullptr;
      o.ld_src = a->ld_src;
      o.y2 = a->y2 ? (void*)(reinterpret_cast<bf16*>(a->y2) + b1 * a->y2_s[0] + b2 * a->y2_s[1]) : nullptr;
      o.ldy2 = a->ldy2;
    } else {
      // lrp input (MCM.py:779-781): [y_hat slots 0..i-1 | y_hat_pre = round(y - mu) + mu] (the quantize_ste
      // value, MCM.py:771-776); y_hat_pre also goes out in f32 (the lrp epilogue's source, read back below
      // after the layer barriers; first touch of those lines by this CU, so no stale L1 copy)
      // the mean stack's output (f32) of problem (0, b2)
      const float* mu = reinterpret_cast<const float*>(a->y) + b2 * a->y_s[1];
      const int ldmu = a->ldy, cc1 = a->cc1, sw = a->ccout[a->cn - 1];
      const bf16* cx1 = reinterpret_cast<const bf16*>(a->cx1) + b2 * a->cs_x1;
      const float* yv = a->yv + b2 * a->cs_yv;
      float* ypre = a->csrc + b2 * a->cs_src;
      const int cld1 = a->cld1, ldyv = a->ldyv, ldp = a->cld_src;
      cin = cc1 + sw;
      const int q = pad32(cin) >> 3, pin = pitch(cin);
      for (int i = tid; i < npix * q; i += NW * 64) {
        const int p = i / q, ch = 8 * (i - p * q);
        const size_t row = (size_t)img * npix + p;
        uint4 v = uint4{0, 0, 0, 0};
        if (ch < cc1) {
          v = *reinterpret_cast<const uint4*>(cx1 + row * cld1 + ch);
        } else if (ch < cin) {
          const int c = ch - cc1;
          f32x4 y0, y1, m0, m1;
          load8f(yv + row * ldyv + c, y0, y1);
          load8f(mu + row * ldmu + c, m0, m1);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y0[e] = rintf(y0[e] - m0[e]) + m0[e];
            y1[e] = rintf(y1[e] - m1[e]) + m1[e];
          }
          store8(ypre + row * ldp + c, y0, y1);
          v = pack8_bf16(y0, y1);
        }
        *reinterpret_cast<uint4*>(lb + p * pin + 2 * ch) = v;
      }
      __syncthreads();
      o.add = a->cadd ? a->cadd + b2 * a->cs_add : nullptr;
      o.ld_add = a->cld_add;
      o.y_f32 = 0;
      o.y = reinterpret_cast<bf16*>(a->cy) + b2 * a->cs_y;
      o.ldy = a->cldy;
      o.src = ypre;
      o.ld_src = ldp;
      o.y2 = a->cy2 ? (void*)(reinterpret_cast<bf16*>(a->cy2) + b2 * a->cs_y2) : nullptr;
      o.ldy2 = a->cldy2;
    }
    const int nl = pass ? a->cn : a->nlayers;
    for (int l = 0; l < nl; ++l) {
      LstkLayer L;
      if (pass == 0) {
        L.w = reinterpret_cast<const bf16*>(a->w[l]) + b1 * a->w_s[l][0] + b2 * a->w_s[l][1];
        L.b = a->bias[l] ? a->bias[l] + b1 * a->b_s[l][0] + b2 * a->b_s[l][1] : nullptr;
        L.cout = a->cout[l];
      } else {
        L.w = reinterpret_cast<const bf16*>(a->cw[l]) + b2 * a->cs_w[l];
        L.b = a->cb[l] + b2 * a->cs_b[l];
        L.cout = a->ccout[l];
      }
      L.cin = cin;
      const bool first = l == 0, last = l + 1 == nl;
      o.route = o.bwd && last && a->racc[0] != nullptr;
      o.ra = a;
      o.rb1 = (int)b1;
      if (pass == 0) {
        o.sp = a->sv_pre[l] && (!last || o.bwd) ? reinterpret_cast<bf16*>(a->sv_pre[l]) + b1 * a->sv_s[l][0] + b2 * a->sv_s[l][1]
                                                : nullptr;
        o.sa = o.sp ? reinterpret_cast<bf16*>(a->sv_act[l]) + b1 * a->sv_s[l][0] + b2 * a->sv_s[l][1] : nullptr;
        o.st = a->sv_t && last ? a->sv_t + b1 * a->sv_t_s[0] + b2 * a->sv_t_s[1] : nullptr;
      } else {
        o.sp = a->csv_pre[l] && !last ? reinterpret_cast<bf16*>(a->csv_pre[l]) + b2 * a->cs_sv[l] : nullptr;
        o.sa = o.sp ? reinterpret_cast<bf16*>(a->csv_act[l]) + b2 * a->cs_sv[l] : nullptr;
        o.st = a->csv_t && last ? a->csv_t + b2 * a->cs_t : nullptr;
      }
#if LSTK_TRACE
      o.trl = 2 + 4 * min(tr_layer, 10);
      lstk_tr_set(o.trl, __builtin_amdgcn_s_memtime());
#endif
      const unsigned in_off = (l & 1) ? (unsigned)BUF : 0u, out_off = (l & 1) ? 0u : (unsigned)BUF;
      const int nfr = (L.cout + 15) >> 4;
      const int nkc = pad32(L.cin) >> 5;
      // (Round 4 measured a host-planned split with finer items -- pairs / singles x pixel chunks of 1..5, chosen
      // per layer to balance the waves -- at 2x the time per launch: ms_3 114.7 vs 63.3 us, profiles/r04/
      // c6_ls_*.log.  Each item streams its weight fragments from L2 for its own pixel chunk, so a chunk of 3
      // fragments or fewer needs >= 46 TB/s of L2 at the MFMA rate, and every item restarts the weight ring.)
      // wave items.  LDS bandwidth binds first: one 1-KiB B read per 16-cycle MFMA on every SIMD is the
      // whole 256 B/clk array, so every wide layer shares each B read between two output fragments
      // (NF = 2); the pixel fragments are split in halves (5 + 4) where that balances the four SIMDs better:
      //   >= 14 output fragments (224): fragment pairs x all pixel fragments (7 items);
      //   8..13 (176, 128): fragment pairs x pixel halves, all first halves dealt before the second ones;
      //   < 8 (80, 32): single fragments x pixel halves.
      const bool halves = nmf > 5;
      if (nfr >= 8) {
        const int ng = (nfr + 1) >> 1;
        if (nfr >= 14 || !halves) {
          for (int it = wave; it < ng; it += NW)
            lstk_dispatch<2, 9, BWD>(nkc, L, first, last, o, img, 2 * it, 0, lb, in_off, out_off, npix, G, lane);
        } else {
          for (int it = wave; it < 2 * ng; it += NW) {
            const int g = it < ng ? it : it - ng;
            if (it < ng) lstk_dispatch<2, 5, BWD>(nkc, L, first, last, o, img, 2 * g, 0, lb, in_off, out_off, npix, G, lane);
            else lstk_dispatch<2, 4, BWD>(nkc, L, first, last, o, img, 2 * g, 5, lb, in_off, out_off, npix, G, lane);
          }
        }
      } else if (!halves) {
        for (int it = wave; it < nfr; it += NW)
          lstk_dispatch<1, 5, BWD>(nkc, L, first, last, o, img, it, 0, lb, in_off, out_off, npix, G, lane);
      } else {
        for (int it = wave; it < 2 * nfr; it += NW) {
          const int f = it < nfr ? it : it - nfr;
          if (it < nfr) lstk_dispatch<1, 5, BWD>(nkc, L, first, last, o, img, f, 0, lb, in_off, out_off, npix, G, lane);
          else lstk_dispatch<1, 4, BWD>(nkc, L, first, last, o, img, f, 5, lb, in_off, out_off, npix, G, lane);
        }
      }
      if (!last) {
        // zero the channel padding [cout, pad32(cout)) the next layer's 32-wide K steps read
        const int cp = pad32(L.cout), pz = pitch(L.cout);
        const int q = (cp - L.cout) >> 3;  // 16-B pieces per row (cout is a multiple of 8)
        if (q > 0)
          for (int i = tid; i < npix * q; i += NW * 64) {
            const int p = i / q, ch = L.cout + 8 * (i - p * q);
            *reinterpret_cast<uint4*>(lb + out_off + p * pz + 2 * ch) = uint4{0, 0, 0, 0};
          }
      }
      cin = L.cout;
#if LSTK_TRACE
      lstk_tr_set(o.trl + 3, __builtin_amdgcn_s_memtime());
      ++tr_layer;
#endif
      __syncthreads();
    }
  }
#if LSTK_TRACE
  lstk_tr_set(47, __builtin_amdgcn_s_memtime());
#endif
}

extern "C" int tmae_lic_stack(const tmae_lic_stack_args* args, void* stream) {
  using namespace lstk;
  TMAE_REQUIRE(args != nullptr, "tmae_lic_stack: args is NULL");
  const tmae_lic_stack_args& a = *args;
  TMAE_REQUIRE(a.G >= 1 && a.G * a.G <= MAXPIX, "tmae_lic_stack: grid %dx%d exceeds %d pixels", a.G, a.G, MAXPIX);
  TMAE_REQUIRE(a.nlayers >= 1 && a.nlayers <= TMAE_LIC_STACK_MAXL, "tmae_lic_stack: %d layers", a.nlayers);
  TMAE_REQUIRE(a.nb1 >= 1 && a.nb2 >= 1 && a.n >= 1, "tmae_lic_stack: batch %d x %d, n %d", a.nb1, a.nb2, a.n);
  const bool bwd = (a.flags & TMAE_LIC_STACK_BWD) != 0;
  TMAE_REQUIRE(a.x1 != nullptr && (a.y != nullptr || bwd), "tmae_lic_stack: x1 / y required");
  if (bwd) {
    TMAE_REQUIRE(!(a.flags & TMAE_LIC_STACK_CHAIN) && !a.addend && !a.lrp_src && !a.x2 && !a.sv_t,
                 "tmae_lic_stack: the backward chain takes no chain / addend / lrp / second source");
    const bool rt = a.racc[0] != nullptr;
    for (int l = 0; l < a.nlayers; ++l)
      TMAE_REQUIRE(a.w[l] && ((rt && l + 1 == a.nlayers) || (a.sv_pre[l] && a.sv_act[l])),
                   "tmae_lic_stack: backward layer %d needs w / sv_pre / sv_act", l);
    if (rt) {
      const int cl = a.cout[a.nlayers - 1];
      // the routed accumulators step by the problem's nb1 index only (racc + b1 * rs)
      TMAE_REQUIRE(a.nb2 <= 1, "tmae_lic_stack: routed accumulators need nb2 == 1 (got %d)", a.nb2);
      TMAE_REQUIRE(a.rlim[0] >= 0 && a.rlim[0] <= a.rlim[1] && a.rlim[1] <= a.rlim[2] && a.rlim[2] == cl &&
                   a.rlim[0] % 4 == 0 && a.rlim[1] % 4 == 0, "tmae_lic_stack: routes %d / %d / %d of %d channels",
                   a.rlim[0], a.rlim[1], a.rlim[2], cl);
      for (int r = 0; r < 3; ++r)
        TMAE_REQUIRE((r == 0 ? a.rlim[0] : a.rlim[r] - a.rlim[r - 1]) == 0 || (a.racc[r] && a.rld[r] % 4 == 0),
                     "tmae_lic_stack: route %d accumulator", r);
    }
  }
  TMAE_REQUIRE(a.c1 >= 0 && a.c2 >= 0 && (a.c2 == 0 || a.x2 != nullptr), "tmae_lic_stack: channels %d + %d", a.c1, a.c2);
  TMAE_REQUIRE(a.c1 % 8 == 0 && a.c2 % 8 == 0 && a.ld1 % 8 == 0 && (a.c2 == 0 || a.ld2 % 8 == 0),
               "tmae_lic_stack: input channels / strides must be multiples of 8");
  TMAE_REQUIRE(pad32(a.c1 + a.c2) <= MAXC, "tmae_lic_stack: %d input channels exceed %d", a.c1 + a.c2, MAXC);
  for (int l = 0; l < a.nlayers; ++l) {
    TMAE_REQUIRE((a.w[l] != nullptr || (l == 0 && a.c1 + a.c2 == 0)) && (a.bias[l] != nullptr || bwd),
                 "tmae_lic_stack: layer %d weights", l);
    TMAE_REQUIRE(a.cout[l] >= 4 && a.cout[l] % 8 == 0, "tmae_lic_stack: layer %d cout %d (multiple of 8)", l, a.cout[l]);
    TMAE_REQUIRE((l + 1 == a.nlayers && (!bwd || a.racc[0])) || pad32(a.cout[l]) <= MAXC,
                 "tmae_lic_stack: layer %d cout %d exceeds %d", l, a.cout[l], MAXC);
  }
  TMAE_REQUIRE(!a.lrp_src || !a.y_f32, "tmae_lic_stack: lrp output is bf16");
  if (a.flags & TMAE_LIC_STACK_CHAIN) {
    TMAE_REQUIRE(a.nb1 == 2 && a.y_f32 && !a.lrp_src && a.cn >= 1 && a.cn <= TMAE_LIC_STACK_MAXL,
                 "tmae_lic_stack: chain needs the 2 x nb2 mean / scale problems with f32 outputs");
    TMAE_REQUIRE(a.ccout[a.cn - 1] == a.cout[a.nlayers - 1] && a.cx1 && a.yv && a.csrc && a.cy,
                 "tmae_lic_stack: chain operands");
    TMAE_REQUIRE(a.cc1 % 8 == 0 && a.cld1 % 8 == 0 && a.ldyv % 4 == 0 && a.cld_src % 4 == 0 && a.ldy % 4 == 0 &&
                 pad32(a.cc1 + a.ccout[a.cn - 1]) <= MAXC, "tmae_lic_stack: chain channels %d + %d", a.cc1,
                 a.ccout[a.cn - 1]);
    for (int l = 0; l < a.cn; ++l)
      TMAE_REQUIRE(a.cw[l] && a.cb[l] && a.ccout[l] % 8 == 0 && (l + 1 == a.cn || pad32(a.ccout[l]) <= MAXC),
                   "tmae_lic_stack: chain layer %d", l);
  }
  if (a.addend) TMAE_REQUIRE(a.ld_add % 4 == 0, "tmae_lic_stack: addend stride %d", a.ld_add);
  for (int l = 0; l < a.nlayers; ++l)
    TMAE_REQUIRE(!a.sv_pre[l] == !a.sv_act[l], "tmae_lic_stack: layer %d keeps pre-activation and output together", l);
  for (int l = 0; l < a.cn && (a.flags & TMAE_LIC_STACK_CHAIN); ++l)
    TMAE_REQUIRE(!a.csv_pre[l] == !a.csv_act[l], "tmae_lic_stack: chain layer %d keeps pre and output together", l);
  TMAE_REQUIRE(!a.sv_t || a.lrp_src, "tmae_lic_stack: sv_t is the lrp stack's pre-tanh value");
  const int nwg = a.n * a.nb1 * a.nb2;
  if (bwd) hipLaunchKernelGGL(lic_stack_kernel<true>, dim3(nwg), dim3(NW * 64), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(lic_stack_kernel<false>, dim3(nwg), dim3(NW * 64), 0, (hipStream_t)stream, a);
  TMAE_LAUNCH_CHECK("tmae_lic_stack");
}

// ================================================================== latent-channel partial sums
// tmae_lic_latent: the first convs' latent part of every slice stack as ONE packed conv (cin <= 384, one image x 16
// output fragments per workgroup).  The halo kernel (conv_halo.h) it replaces stages the weight slab of every
// (64-channel chunk, tap) step through LDS behind a barrier: operands of both sides read from LDS and a barrier per
// step.  Here, as in lic_stack, the image's input rows stay in LDS for the whole K sweep and every wave streams its
// own two weight fragments per K-step from L2 into registers: no barrier inside the sweep, B reads shared by two
// MFMAs.  Summation order per output: taps outer, 32-channel steps inner.
namespace llat {
constexpr int NW = 8, FPW = 2 * NW;  // fragments per workgroup (one pair per wave)
constexpr int MAXCIN = 384;
constexpr unsigned PMAX = lstk::pitch(MAXCIN);
constexpr unsigned ZOFF = lstk::MAXPIX * PMAX;  // 16 zero rows past the 144 input rows
constexpr unsigned TMASK = ZOFF + 16 * PMAX;
constexpr int LDS_BYTES = TMASK + 320;
}  // namespace llat
__device__ __forceinline__ constexpr unsigned llat_zoff() { return llat::ZOFF; }
__device__ __forceinline__ constexpr unsigned llat_tmask() { return llat::TMASK; }

// one wave: output fragments f0, f0 + 1 x all 9 pixel fragments over the 9 x NKC K-steps.  The tap loop is rolled
// (108 unrolled steps at cin 384 left the ring arrays in scratch); inside a tap the NKC steps are unrolled, and
// with D | NKC the A ring's slots stay static registers across taps (step s in slot (s mod NKC) mod D).
// epilogue operands of one problem: output (f32 or bf16, rows ldy apart) starting at the problem's first fragment's
// column, optional bias over those columns, optional GELU
struct LlatOut {
  void* y;
  int ldy, bf, act;
  const float* bias;
};

template <int NKC>
__device__ __forceinline__ void llat_item(const bf16* w, int nfr, long long blk, int f0, int fcol, bool two,
                                          const unsigned char* lb, unsigned pin, int G, int npix, int img,
                                          const LlatOut& o, int lane) {
  constexpr int MF = 9, NS = 9 * NKC;
  constexpr int D = NKC % 4 == 0 ? 4 : NKC % 3 == 0 ? 3 : NKC % 2 == 0 ? 2 : (NKC <= 7 ? NKC : 1);
  asm volatile("" : "+v"(lane));
  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[2][MF];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < MF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned sstride = (unsigned)nfr * 512u;
  const bf16* wl[2];
  bf16x8 ar[D][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int f = two || i == 0 ? f0 + i : f0;  // a lone last fragment: the pair's second half re-reads the first
    const int b = f / nfr, fi = f - b * nfr;
    wl[i] = w + b * blk + ((size_t)fi * 64 + lane) * 8;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      ar[d][i] = *reinterpret_cast<const bf16x8*>(wl[i]);
      wl[i] += sstride;
    }
  }
  unsigned tmask[MF];
#pragma unroll
  for (int j = 0; j < MF; ++j) tmask[j] = *reinterpret_cast<const unsigned short*>(lb + llat_tmask() + 2 * (16 * j + fr));
  auto row = [&](int t, int j) -> unsigned {
    const int p = 16 * j + fr, sh = (t / 3 - 1) * G + (t % 3 - 1);
    const unsigned r = (unsigned)(p + sh);
    return ((tmask[j] >> t) & 1u ? r * pin : llat_zoff() + (r & 15u) * pin) + 16u * fq;
  };
  bf16x8 bv[2][MF];
  unsigned rb[MF];
#pragma unroll
  for (int j = 0; j < MF; ++j) {
    rb[j] = row(0, j);
    bv[0][j] = *reinterpret_cast<const bf16x8*>(lb + rb[j]);
  }
  for (int t = 0; t < 9; ++t) {
    unsigned rn[MF];
#pragma unroll
    for (int j = 0; j < MF; ++j) rn[j] = row(t + 1 < 9 ? t + 1 : t, j);
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc) {
      if (kc + 1 < NKC) {
#pragma unroll
        for (int j = 0; j < MF; ++j) bv[(kc + 1) & 1][j] = *reinterpret_cast<const bf16x8*>(lb + rb[j] + 64u * (kc + 1));
      } else if (t + 1 < 9) {
#pragma unroll
        for (int j = 0; j < MF; ++j) bv[(kc + 1) & 1][j] = *reinterpret_cast<const bf16x8*>(lb + rn[j]);
      }
      bf16x8 a0[2];
      const bool more = t * NKC + kc + D < NS;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        a0[i] = ar[kc % D][i];
        if (more) {
          ar[kc % D][i] = *reinterpret_cast<const bf16x8*>(wl[i]);
          wl[i] += sstride;
        }
      }
#pragma unroll
      for (int j = 0; j < MF; ++j)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], bv[kc & 1][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (NKC & 1) {  // odd step count per tap: the next tap's first B fragments went to buffer 1
#pragma unroll
      for (int j = 0; j < MF; ++j) bv[0][j] = bv[1][j];
    }
#pragma unroll
    for (int j = 0; j < MF; ++j) rb[j] = rn[j];
  }
  // lane: columns fcol + 16 i + 4 fq .. + 3 (fragment f0 + i) of pixel 16 j + fr
  f32x4 bias[2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    bias[i] = o.bias ? load4f(o.bias + fcol + 16 * (two ? i : 0) + 4 * fq) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < MF; ++j) {
    const int p = 16 * j + fr;
    if (p >= npix) continue;
    const size_t at = ((size_t)img * npix + p) * o.ldy + fcol + 4 * fq;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (i == 1 && !two) break;
      f32x4 v = acc[i][j] + bias[i];
      if (o.act == TMAE_ACT_GELU) {
        const f32x2 lo = gelu2_bf16out(v.xy), hi = gelu2_bf16out(v.zw);
        v = f32x4{lo.x, lo.y, hi.x, hi.y};
      }
      if (o.bf) store4(reinterpret_cast<bf16*>(o.y) + at + 16 * i, v);
      else store4(reinterpret_cast<float*>(o.y) + at + 16 * i, v);
    }
  }
}

template <int NKC>
__global__ void __launch_bounds__(llat::NW * 64) lic_latent_kernel(tmae_lic_latent_args a) {
  using namespace llat;
  __shared__ __attribute__((aligned(16))) uint4 lds[LDS_BYTES / 16];
  unsigned char* lb = reinterpret_cast<unsigned char*>(lds);
  const int n = a.n, G = a.G, npix = G * G, cin = 32 * NKC;
  const int t = xcd_remap(blockIdx.x, gridDim.x);  // tile-major: an XCD's run shares its tiles' weights in L2
  const int tile = t / n, img = t - tile * n, prob = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const unsigned pin = lstk::pitch(cin);
  for (int i = tid; i < 16 * (int)pin / 16; i += NW * 64) reinterpret_cast<uint4*>(lds)[ZOFF / 16 + i] = uint4{0, 0, 0, 0};
  for (int p = tid; p < 160; p += NW * 64) {
    unsigned m = 0;
    if (p < npix) {
      const int py = p / G, px = p - py * G;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int yy = py + k / 3 - 1, xx = px + k % 3 - 1;
        m |= ((unsigned)yy < (unsigned)G && (unsigned)xx < (unsigned)G) ? (1u << k) : 0u;
      }
    }
    *reinterpret_cast<unsigned short*>(lb + TMASK + 2 * p) = (unsigned short)m;
  }
  {
    const bf16* x = reinterpret_cast<const bf16*>(a.x[prob]);
    constexpr int q = 4 * NKC;  // 16-B pieces per row
    for (int i = tid; i < npix * q; i += NW * 64) {
      const int p = i / q, ch = 8 * (i - p * q);
      *reinterpret_cast<uint4*>(lb + p * pin + 2 * ch) =
          *reinterpret_cast<const uint4*>(x + ((size_t)img * npix + p) * a.ldx + ch);
    }
  }
  __syncthreads();
  const int fr0 = a.f_lo + tile * FPW + 2 * wave;  // this wave's first fragment, relative to the problem's
  if (fr0 >= a.f_hi) return;  // past this launch's fragments (no barrier follows)
  LlatOut o;
  o.ldy = a.ldy;
  o.bf = a.y_bf16;
  o.act = a.act;
  o.bias = a.bias[prob];
  o.y = a.y_bf16 ? (void*)(reinterpret_cast<bf16*>(a.y) + a.y_s[prob]) : (void*)(a.y + a.y_s[prob]);
  llat_item<NKC>(reinterpret_cast<const bf16*>(a.w), a.nfr, a.blk, a.f_off[prob] + fr0, 16 * fr0, fr0 + 1 < a.f_hi, lb,
                 pin, G, npix, img, o, lane);
}

extern "C" int tmae_lic_latent(const tmae_lic_latent_args* args, void* stream) {
  TMAE_REQUIRE(args != nullptr, "tmae_lic_latent: args is NULL");
  const tmae_lic_latent_args& a = *args;
  TMAE_REQUIRE(a.G >= 1 && a.G * a.G <= lstk::MAXPIX, "tmae_lic_latent: grid %dx%d", a.G, a.G);
  TMAE_REQUIRE(a.cin >= 32 && a.cin % 32 == 0 && a.cin <= llat::MAXCIN, "tmae_lic_latent: cin %d (multiple of 32, <= %d)",
               a.cin, llat::MAXCIN);
  TMAE_REQUIRE(a.nb >= 1 && a.nb <= TMAE_LIC_LATENT_MAXP && a.n >= 1, "tmae_lic_latent: %d problems, %d images", a.nb,
               a.n);
  TMAE_REQUIRE(a.w && a.y && a.ldx % 8 == 0 && a.ldx >= a.cin, "tmae_lic_latent: operands / strides");
  TMAE_REQUIRE(a.nfr >= 1 && a.f_lo >= 0 && a.f_hi > a.f_lo && a.f_lo % 2 == 0, "tmae_lic_latent: fragments [%d, %d) "
               "of blocks of %d (f_lo even)", a.f_lo, a.f_hi, a.nfr);
  TMAE_REQUIRE(a.blk >= 9LL * (a.cin / 32) * a.nfr * 512 || a.f_off[0] + a.f_hi <= a.nfr, "tmae_lic_latent: block stride");
  TMAE_REQUIRE(a.act == TMAE_ACT_NONE || a.act == TMAE_ACT_GELU, "tmae_lic_latent: act %d", a.act);
  TMAE_REQUIRE(a.ldy % 4 == 0 && (a.ldy >= 16 * a.f_hi), "tmae_lic_latent: ldy %d", a.ldy);
  for (int j = 0; j < a.nb; ++j)
    TMAE_REQUIRE(a.x[j] && a.f_off[j] >= 0 && a.y_s[j] % 4 == 0, "tmae_lic_latent: problem %d", j);
  const int ntile = (a.f_hi - a.f_lo + llat::FPW - 1) / llat::FPW;
  const dim3 grid(a.n * ntile, a.nb);
  hipStream_t st = (hipStream_t)stream;
  switch (a.cin / 32) {
#define LLAT_CASE(K) \
  case K: hipLaunchKernelGGL(lic_latent_kernel<K>, grid, dim3(llat::NW * 64), 0, st, a); break;
    LLAT_CASE(1) LLAT_CASE(2) LLAT_CASE(3) LLAT_CASE(4) LLAT_CASE(5) LLAT_CASE(6)
    LLAT_CASE(7) LLAT_CASE(8) LLAT_CASE(9) LLAT_CASE(10) LLAT_CASE(11) LLAT_CASE(12)
#undef LLAT_CASE
    default: break;
  }
  TMAE_LAUNCH_CHECK("tmae_lic_latent");
}
