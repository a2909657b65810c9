/*
 * tmae.h — C ABI of libtmae.so, the MI355X (gfx950) kernels behind the TextMAE MCM hot path.
 *
 * The reference path is pure Python on PyTorch + compressai + timm (no native code of its own).
 * Each entry point below replaces the reference computation cited next to it; the Python host
 * (textmae-image-compression_amd/mcm.py) calls these through ctypes exactly where the reference's
 * nn.Module code runs (INTEGRATION.md shows the binding).
 *
 * Conventions
 *   - all pointers are device pointers (hipMalloc / torch caching allocator); the library never
 *     allocates, never synchronises, and enqueues on `stream` (a hipStream_t, NULL = default);
 *   - `dtype` selects the MFMA operand type: TMAE_F32 (exact f32 MFMA, parity path) or TMAE_BF16
 *     (bf16 operands, f32 accumulate, throughput path); accumulation, residual stream, entropy
 *     models and likelihoods are always f32;
 *   - activations are row-major "token" matrices [rows][channels]; LIC feature maps are NHWC;
 *     likelihood outputs are NCHW like the reference's tensors;
 *   - return 0 on success, TMAE_EINVAL for a bad shape/argument, TMAE_EHIP for a launch error;
 *     tmae_last_error_string() describes the last failure on the calling thread.
 */
#ifndef TMAE_H
#define TMAE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TMAE_ABI_VERSION 1

enum { TMAE_OK = 0, TMAE_EINVAL = 1, TMAE_EHIP = 2 };
enum { TMAE_F32 = 0, TMAE_BF16 = 1 };
enum { TMAE_ACT_NONE = 0, TMAE_ACT_GELU = 1, TMAE_ACT_RELU = 2 /* tmae_conv3x3 plain stores only (VGG16) */ };

const char* tmae_last_error_string(void);
int tmae_abi_version(void);

/* ---- masking -------------------------------------------------------------------------------
 * MCM.get_ids_shuffle (models/Compression/MCM.py:364-423) + the argsort / keep-slice of
 * MCM.random_masking (MCM.py:579-583).  scores [n][L] f32 -> ids_shuffle, ids_restore [n][L] i64.
 * Bit-exact with the reference.  sum_lanes = torch CPU float-sum vector width (8 on x86 AVX2/512
 * builds).  Raises TMAE_EINVAL for K > L exactly where MCM.py:374-376 raises. */
int tmae_ids_shuffle(const float* scores, int64_t* ids_shuffle, int64_t* ids_restore, int n, int L, int K,
                     int sum_lanes, void* stream);

/* ---- transformer (timm 0.4.5 Block / PatchEmbed, used at MCM.py:300-348, 615-632, 657-686) ---- */

/* LayerNorm(eps) over f32 rows; source row = (r / row_group) * group_stride + row_offset + r % row_group
 * (drops cls rows without a copy: MCM.py:631-632).  y is f32 or bf16 (out_dtype). */
int tmae_layernorm_fwd(const float* x, const float* gamma, const float* beta, void* y, int rows, int D,
                       int row_group, int group_stride, int row_offset, float eps, int out_dtype, void* stream);

/* y[M][N] = act(x[M][K] · w[N][K]^T + bias).  x is f32 (x_f32=1) or dtype; y is f32 (y_f32=1) or dtype.
 * nn.Linear / 1x1 Conv2d (g_a, MCM.py:77-93) / 1x1 ConvTranspose2d with pre-transposed weight (g_s,
 * MCM.py:96-112).  Same row remap as tmae_layernorm_fwd.  y32 (optional): second f32 copy of the output
 * (g_a's last layer feeds the f32 Gaussian likelihood and the bf16 h_a convs). */
int tmae_linear_fwd(const void* x, int x_f32, int ldx, int row_group, int group_stride, int row_offset,
                    const void* w, const float* bias, void* y, int y_f32, int ldy, float* y32, int ld32, int M, int N,
                    int K, int act, int dtype, void* stream);

/* resid[M][N] += x[M][K] · w[N][K]^T + bias   (Attention.proj / Mlp.fc2 + the Block residual adds) */
int tmae_linear_residual_fwd(const void* x, int ldx, const void* w, const float* bias, float* resid, int ldr,
                             int M, int N, int K, int dtype, void* stream);

/* PatchEmbed conv16/s16 + pos_embed + masking gather, over the KEPT patches only
 * (MCM.py:615-621 then the gather at 585-586): tokens [n][keep+1][D], rows 1..keep written;
 * w = proj.weight viewed [D][C*P*P], each row zero-padded to a multiple of 8 values when C*P*P is not
 * (patch 14: 588 -> 592).  Any patch size dividing the image; rows of P % 8 != 0 gather per value. */
int tmae_patch_embed_fwd(const float* imgs, const int64_t* ids_shuffle, const void* w, const float* bias,
                         const float* pos, float* tokens, int n, int C, int H, int W, int patch, int D, int L,
                         int keep, int dtype, void* stream);

/* the same projection over kept patches gathered beforehand by tmae_patch_gather (patches [n*keep][Kw] in the
 * operand dtype, Kw = C*P*P when P % 8 == 0): the LDS-DMA GEMM instead of the converting register path, same
 * MFMA k-order (same tokens). */
int tmae_patch_embed_gathered(const void* patches, const int64_t* ids_shuffle, const void* w, const float* bias,
                              const float* pos, float* tokens, int n, int Kw, int D, int L, int keep, int dtype,
                              void* stream);

/* tokens[b][0] = cls_token + pos[0]  (MCM.py:624-626) */
int tmae_cls_rows(float* tokens, const float* cls, const float* pos, int n, int rows_per_img, int D, void* stream);

/* Fused multi-head attention over qkv [B*T][3*H*dh] (timm layout (3, H, dh)) -> out [B*T][H*dh];
 * softmax((q k^T) * scale) v, dh in {32, 64, 80} (80: ViT-H, models_mae.py:239-244), T <= 512. */
int tmae_mha_fwd(const void* qkv, void* out, int B, int T, int H, int dh, float scale, int dtype, void* stream);

/* qkv Linear + multi-head attention in one launch (bf16 inference; timm Attention qkv + core, MCM.py:629-630,
 * 678-679): out [B*T][H*dh] = attention of [q | k | v] = x W_qkv^T + b_qkv, x [B*T][H*dh] bf16, W_qkv
 * [3*H*dh][H*dh] bf16 (nn.Linear layout), b_qkv [3*H*dh] f32.  Q / K / V stay in LDS (no qkv tensor in HBM);
 * output bit-identical to tmae_linear_fwd(qkv) + tmae_mha_fwd.  Shapes with a fused kernel:
 * tmae_qkv_attn_supported (dh 64 with T in (128, 160] or (64, 96]; dh 32 with T in (256, 288], H even). */
int tmae_qkv_attn_supported(int T, int H, int dh);
int tmae_qkv_attn_fwd(const void* x, const void* w_qkv, const float* b_qkv, void* out, int B, int T, int H, int dh,
                      float scale, int dtype, void* stream);

/* decoder_embed + mask-token unshuffle + decoder_pos_embed (MCM.py:657-675):
 * x [n*ntok][Din] -> out [n][L+1][D]; token k -> row 0 (k=0) or 1 + ids_shuffle[b][k-1].
 * ntok = K for MCM (cls already dropped: the reference's off-by-one), K+1 for MAE. */
int tmae_decoder_embed_fwd(const void* x, int x_f32, const void* w, const float* bias, const float* pos,
                           const int64_t* ids_shuffle, float* out, int n, int ntok, int L, int Din, int D,
                           int dtype, void* stream);
/* the rows the kept tokens do not cover: mask_token + pos (MCM.py:660-664) */
int tmae_mask_rows(float* out, const float* mask_token, const float* pos, const int64_t* ids_shuffle, int n,
                   int L, int ntok, int D, void* stream);

/* decoder_pred + drop cls + unpatchify (MCM.py:683-686, 524-546, 795-797): x [n*L][Din] (rows 1..L of
 * the decoder, cls excluded) -> imgs [n][C][H][W] f32 */
int tmae_decoder_pred_fwd(const void* x, const void* w, const float* bias, float* imgs, int n, int L, int Din,
                          int C, int H, int W, int patch, int dtype, void* stream);
/* same computation with the weight rows and bias in channel-planar order, row (c*patch + py)*patch + px
 * (the reference's row (py*patch + px)*C + c; the inference executor permutes them once per weight
 * version); patch % 8 == 0. Every lane stores 8 consecutive pixels of one image row. */
int tmae_decoder_pred_cp_fwd(const void* x, const void* w, const float* bias, float* imgs, int n, int L, int Din,
                             int C, int H, int W, int patch, int dtype, void* stream);

/* ---- learned-image-compression stack (MCM.py:729-792), NHWC f32 feature maps ------------------ */

/* Batched 3x3 conv, padding 1 (compressai conv3x3 / nn.Conv2d(k=3, p=1), MCM.py:115-293) as an implicit
 * GEMM.  Inputs are NHWC in the operand dtype; channels [0,c1) come from x1 and [c1,c1+c2) from x2
 * (torch.cat without a copy).  w = [cout][3][3][c1+c2].  nb1*nb2 independent problems run in one
 * launch: problem b = b1*nb2 + b2 offsets every pointer by b1*s1 + b2*s2 elements.
 * Epilogue: y = act(acc + bias + addend) (addend optional: precomputed partial sums), optional f32 copy
 * y32; pixel_shuffle=1 -> subpel_conv3x3 r=2 (output [n][2H][2W][cout/4]); lrp_src set -> the last
 * lrp_transform conv: y (and y2) = lrp_src + 0.5*tanh(acc + bias)  (MCM.py:779-784). */
typedef struct tmae_conv_args {
  const void* x1; int c1, ld1; long long x1_s1, x1_s2;
  const void* x2; int c2, ld2; long long x2_s1, x2_s2;
  int n, H, W, stride;
  const void* w; long long w_s1, w_s2;
  const float* bias; long long b_s1, b_s2;
  int cout, act, pixel_shuffle;
  void* y; int y_f32, ldy; long long y_s1, y_s2;
  float* y32; int ld32; long long y32_s1, y32_s2;
  const float* addend; int ld_add; long long a_s1, a_s2;
  const float* lrp_src; int ld_src; long long src_s1, src_s2;
  void* y2; int ldy2; long long y2_s1, y2_s2;
  int nb1, nb2;
  /* training: optional pre-activation copy (GELU input; the last lrp conv's pre-tanh value, f32) in the
   * output's dtype and layout (pixel-shuffled for subpel convs), rows ldp apart (lrp) */
  void* pre; int ldp; long long pre_s1, pre_s2;
} tmae_conv_args;
int tmae_conv3x3(const tmae_conv_args* args, int dtype, void* stream);

/* A whole slice-transform stack -- cc_transform_mean / cc_transform_scale / lrp_transform[i]
 * (MCM.py:165-293 applied at MCM.py:761-784): `nlayers` 3x3 convs with GELU between them -- for
 * nb1 x nb2 problems x n images over a G x G grid (G*G <= 144), bf16 operands, one workgroup per
 * (problem, image) with the activations resident in LDS (every intermediate <= 224 channels).
 * Layer-0 input: channels [0, c1) of x1 and [c1, c1 + c2) of x2 (NHWC rows ld1 / ld2 apart).
 * w[l]: weights packed by the caller in MFMA fragment order [tap 9][k-step round32(cin)/32][cout
 * fragment round16(cout)/16][lane 64][8], zero-padded (textmae_amd.ops.pack_lic_stack_weight);
 * bias[l]: f32 [cout].  addend (optional, f32, rows ld_add apart) is added to layer 0's output before
 * its GELU (the latent-channel partial sums).  Last layer: y = acc + bias (f32 if y_f32, else bf16),
 * or with lrp_src: y (and y2 if set) = lrp_src + 0.5 tanh(acc + bias) in bf16.  Every operand has
 * per-problem element strides {s1, s2} for problem (b1, b2). */
#define TMAE_LIC_STACK_MAXL 5
typedef struct tmae_lic_stack_args {
  int n, G, nb1, nb2, nlayers;
  const void* x1; int c1, ld1; long long x1_s[2];
  const void* x2; int c2, ld2; long long x2_s[2];
  const void* w[TMAE_LIC_STACK_MAXL]; long long w_s[TMAE_LIC_STACK_MAXL][2];
  const float* bias[TMAE_LIC_STACK_MAXL]; long long b_s[TMAE_LIC_STACK_MAXL][2];
  int cout[TMAE_LIC_STACK_MAXL];
  const float* addend; int ld_add; long long a_s[2];
  void* y; int y_f32, ldy; long long y_s[2];
  const float* lrp_src; int ld_src; long long src_s[2];
  void* y2; int ldy2; long long y2_s[2];
  int flags; /* TMAE_LIC_STACK_CHAIN */
  /* TMAE_LIC_STACK_CHAIN: problems (0, b2) of the nb1 x nb2 = 2 x nb2 launch (slice b2's mean stack;
   * (1, b2) its scale stack) go on with that slice's lrp stack in the same workgroup (MCM.py:771-784):
   * y_hat_pre = round(y - mu) + mu from yv (f32, rows ldyv apart) and the mean stack's f32 output mu, also
   * written to csrc (f32, rows cld_src apart); lrp input = [cx1 channels 0..cc1 | y_hat_pre];
   * cy (and cy2, optional) = y_hat_pre + 0.5 tanh(lrp), bf16.  cw / cb / ccout: the lrp layers (packed as w),
   * cadd: its layer-0 addend.  The Gaussian likelihood of the slice is left to the caller. */
  int cn; const void* cw[TMAE_LIC_STACK_MAXL]; const float* cb[TMAE_LIC_STACK_MAXL]; int ccout[TMAE_LIC_STACK_MAXL];
  const void* cx1; int cc1, cld1;
  const float* yv; int ldyv;
  const float* cadd; int cld_add;
  float* csrc; int cld_src;
  void* cy; int cldy;
  void* cy2; int cldy2;
  /* chain operands of problem (0, b2) are offset by b2 * these element strides (batched slices) */
  long long cs_x1, cs_yv, cs_src, cs_add, cs_y, cs_y2, cs_w[TMAE_LIC_STACK_MAXL], cs_b[TMAE_LIC_STACK_MAXL];
  /* training forward (what the HIP backward reads, mcm_train.py): for every layer l but the last, the
   * pre-activation (acc + bias [+ addend]) sv_pre[l] and the GELU output sv_act[l], bf16 [n*G*G][cout[l]] per
   * problem at element strides sv_s[l]; an lrp stack's last layer also writes sv_t = the pre-tanh value, f32
   * [n*G*G][cout] at strides sv_t_s.  Chain: the lrp pass's csv_pre / csv_act / csv_t, problem (0, b2) offset by
   * b2 * cs_sv[l] / cs_t.  NULL: not written (inference). */
  void* sv_pre[TMAE_LIC_STACK_MAXL]; void* sv_act[TMAE_LIC_STACK_MAXL]; long long sv_s[TMAE_LIC_STACK_MAXL][2];
  float* sv_t; long long sv_t_s[2];
  void* csv_pre[TMAE_LIC_STACK_MAXL]; void* csv_act[TMAE_LIC_STACK_MAXL]; long long cs_sv[TMAE_LIC_STACK_MAXL];
  float* csv_t; long long cs_t;
  /* TMAE_LIC_STACK_BWD with racc[0] set: the last layer is the stack's first conv's input gradient, routed by
   * consecutive channel ranges [0, rlim[0]), [rlim[0], rlim[1]), [rlim[1], rlim[2]) into the f32 accumulators
   * racc[r] (rows rld[r] apart, +=; problem b1 at b1 * rs[r] elements) instead of GELU' and sv_act -- the
   * problems must not share an accumulator */
  float* racc[3]; int rld[3]; int rlim[3]; long long rs[3];
} tmae_lic_stack_args;
#define TMAE_LIC_STACK_CHAIN 1
/* TMAE_LIC_STACK_BWD (training backward, mcm_train.py): the stack's data-gradient chain through LDS.  x1 = the
 * gradient of the stack's output (channels [0, c1)); layer l is the transposed conv of forward layer L-1-l
 * (weights packed transposed and tap-flipped, textmae_amd.ops.pack_lic_stack_weight_t), cout[l] its output
 * channels; its epilogue multiplies by GELU'(sv_pre[l]) (the forward's saved bf16 pre-activation of those
 * channels) and writes the result, bf16, to sv_act[l] (the weight gradient's operand; strides sv_s[l]) and, but
 * for the last layer, into LDS as the next layer's input.  No bias, addend, lrp, chain or y. */
#define TMAE_LIC_STACK_BWD 2
int tmae_lic_stack(const tmae_lic_stack_args* args, void* stream);

/* A stride-1 3x3 conv over G x G grids (G*G <= 144, zero padding) with each image's input resident in LDS and
 * the weights streamed from L2 into registers (lic_stack.hip): the latent-channel partial sums of the slice
 * stacks' first convs (mcm.py _Executor._slices / mcm_train _slices_fwd_fused; MCM.py:761-781 restricted to
 * the first `cin` = latent_means / latent_scales channels of the torch.cat), and the 12x12 convs of h_a
 * (layers 0-1, MCM.py:115-134) and h_s (last layer, MCM.py:136-162).  For problem j < nb (<= 4), relative
 * fragment r in [f_lo, f_hi) (global fragment f = f_off[j] + r):
 *   y_j[row][16 r + c] = act(bias_j[16 r + c] + sum_{tap, ci < cin} W_f[c][ci][tap] x_j[row shifted][ci])
 * with y_j = y + y_s[j] elements (f32, or bf16 when y_bf16; rows ldy apart), bias_j optional (f32), act
 * TMAE_ACT_NONE / _GELU.  w: blocks of nfr fragments, block b = f / nfr at element b * blk, each packed in
 * tmae_lic_stack's order [tap 9][k-step cin/32][fragment nfr][lane 64][8] (ops.pack_lic_stack_weight).
 * x_j: bf16 NHWC rows ldx apart, cin a multiple of 32 and <= 384; f_lo even.  One workgroup = one image x 16
 * fragments. */
#define TMAE_LIC_LATENT_MAXP 4
typedef struct tmae_lic_latent_args {
  int n, G, cin, nb;
  const void* x[TMAE_LIC_LATENT_MAXP]; int ldx;
  const void* w; int nfr; long long blk;
  int f_off[TMAE_LIC_LATENT_MAXP]; int f_lo, f_hi;
  float* y; int ldy;
  long long y_s[TMAE_LIC_LATENT_MAXP];
  const float* bias[TMAE_LIC_LATENT_MAXP];
  int act, y_bf16;
} tmae_lic_latent_args;
int tmae_lic_latent(const tmae_lic_latent_args* args, void* stream);

/* GaussianConditional likelihood + y_hat quantisation for `nslices` consecutive slices of width sw
 * (MCM.py:767-776): lik[NCHW channel yoff + j*sw + c] = GC(y~, max(sigma, .11), mu), LowerBound 1e-9;
 * yhat (dtype yhat_dtype, optional) and yhat32 (f32, optional) [pixel][channel] = round(y - mu) + mu.
 * noise (NCHW like lik) selects the training-mode y~ = y + noise. */
int tmae_gc_slices_fwd(const float* y, int ldy, int yoff, const float* mu, const float* sigma, long long ms_stride,
                       int ld_ms, const float* noise, float* lik, int Mtot, void* yhat, int yhat_dtype, int ld_yhat,
                       float* yhat32, int ld32, int n, int HW, int nslices, int sw, void* stream);

/* compressai EntropyBottleneck parameters (filters = (3, 3, 3, 3)), all f32 device pointers */
typedef struct tmae_eb_params {
  const float* matrix[5]; /* _matrix0 [C][3][1], _matrix1..3 [C][3][3], _matrix4 [C][1][3] */
  const float* bias[5];   /* _bias0..3 [C][3][1], _bias4 [C][1][1] */
  const float* factor[4]; /* _factor0..3 [C][3][1] */
  const float* quantiles; /* [C][1][3] */
} tmae_eb_params;

/* EntropyBottleneck forward likelihood (MCM.py:741) + z_hat = round(z - median) + median
 * (MCM.py:742-744).  z, zhat NHWC [n*HW][C] (zhat in zhat_dtype); lik, noise NCHW.
 * table: device scratch C*59 f32. */
int tmae_eb_likelihood_fwd(const float* z, const tmae_eb_params* params, const float* noise, float* lik,
                           void* zhat, int zhat_dtype, float* table, int n, int C, int HW, void* stream);

/* CompressionModel.aux_loss (utils/engine.py:79): out[0] = sum |f(quantiles) - target| */
int tmae_eb_aux_loss(const tmae_eb_params* params, const float* target, float* out, float* table, int C,
                     void* stream);

/* GaussianConditional.forward, elementwise (same layout for all tensors) */
int tmae_gc_likelihood_fwd(const float* x, const float* scales, const float* means, const float* noise,
                           float* x_tilde, float* lik, int total, float scale_bound, void* stream);

/* RateDistortionLoss bpp (models/Compression/loss/rd_loss.py:19-20): out[0] = (sum log y_lik + sum log z_lik)
 * / (-ln2 * num_pixels), deterministic two-pass f64 reduction.  work: >= 512 doubles of device scratch. */
int tmae_bpp_sum(const float* y_lik, long long ny, const float* z_lik, long long nz, double* work, float* out,
                 double num_pixels, void* stream);

/* layout helper: NHWC (channel stride ldx) -> NCHW */
int tmae_nhwc_to_nchw(const float* x, int ldx, float* y, int n, int C, int HW, void* stream);

/* training-set loader sample (training.py:115-129, utils/dataloader.py:58-61: ToTensor + Normalize) on
 * device-resident uint8 HWC images [nsrc][H][W][3]: out[b] = (crop / 255 - mean) / std, NCHW f32 [B][3][S][S];
 * crops [B][3] int32 device = (image, top, left), each crop inside its image (caller's contract).
 * mean / std: 3 host floats each. */
int tmae_crop_normalize_u8(const unsigned char* src, int nsrc, int H, int W, const int* crops, int B, int S,
                           const float* mean, const float* std, float* out, void* stream);

/* ---------------------------------------------------------------- MaskedAutoencoderViT (models/MAE/models_mae.py)
 * random_masking (123-148): ids_shuffle = stable ascending argsort(noise) per row, ids_restore = its
 * inverse, mask[b][l] = 1 where rank >= len_keep (mask may be NULL).  L <= 2048. */
int tmae_mae_masking(const float* noise, int64_t* ids_shuffle, int64_t* ids_restore, float* mask, int n, int L,
                     int len_keep, void* stream);

/* forward_loss (198-214): mean over masked patches of mean((pred - patchify(imgs))^2), per-patch normalised
 * targets if norm_pix_loss.  pred [n*L][P*P*C] f32, imgs NCHW f32 (H == W), work >= 1024 doubles, out[0]. */
int tmae_mae_loss(const float* pred, const float* imgs, const int64_t* ids_restore, int n, int C, int H, int W, int P,
                  int len_keep, int norm_pix_loss, double* work, float* out, void* stream);

/* forward_loss backward (autograd of models_mae.py:212-214): out[n*L][P*P*C] = dloss[0] * mask * 2 (pred - target)
 * / (P*P*C * n * (L - len_keep)) (+ dpred_in when non-NULL), in out_dtype (TMAE_F32 / TMAE_BF16).  dloss may be
 * NULL (no loss gradient: out = dpred_in or zeros). */
int tmae_mae_loss_bwd(const float* pred, const float* imgs, const int64_t* ids_restore, int n, int C, int H, int W,
                      int P, int len_keep, int norm_pix_loss, const float* dloss, const float* dpred_in, void* out,
                      int out_dtype, void* stream);

/* ---------------------------------------------------------------- entropy coding, device side
 * (MCM.compress / decompress, MCM.py:805-968; compressai semantics restated, see rans.cpp) */

/* MCM.compress slice step (MCM.py:864-872): tmae_gc_slices_fwd's eval outputs (y_hat, likelihood) plus
 * symbols = round(y - mu) and indexes = build_indexes(sigma) against scale_table[nscale], both written in
 * the coder's order [slice][image][channel][pixel] starting at slice 0 of this launch. */
int tmae_gc_slices_code(const float* y, int ldy, int yoff, const float* mu, const float* sigma, long long ms_stride,
                        int ld_ms, float* lik, int Mtot, void* yhat, int yhat_dtype, int ld_yhat, float* yhat32,
                        int ld32, int n, int HW, int nslices, int sw, int* symbols, int* indexes,
                        const float* scale_table, int nscale, void* stream);

/* GaussianConditional.build_indexes (MCM.py:938) for nslices slices of sigma rows (layout as above) */
int tmae_gc_indexes(const float* sigma, long long ms_stride, int ld_ms, int n, int HW, int nslices, int sw,
                    const float* scale_table, int nscale, float scale_bound, int* indexes, void* stream);

/* GaussianConditional.dequantize (MCM.py:946): y_hat = symbols + mu into channels yoff.. of y_hat rows */
int tmae_gc_dequantize(const int* symbols, const float* mu, long long ms_stride, int ld_ms, int n, int HW,
                       int nslices, int sw, int yoff, void* yhat, int yhat_dtype, int ld_yhat, float* yhat32, int ld32,
                       void* stream);

/* GaussianConditional.update (update_scale_table): pmf[n][max_length], tail[n] for the CDF builder */
int tmae_gc_pmf(const float* scale_table, const int* pmf_center, int n, int max_length, float* pmf, float* tail,
                void* stream);

/* EntropyBottleneck.update: pmf[C][max_length] at pmf_start[c] + j, tail[C] */
int tmae_eb_pmf(const tmae_eb_params* params, float* table, const float* pmf_start, int C, int max_length, float* pmf,
                float* tail, void* stream);

/* EntropyBottleneck.compress / decompress value maps: symbols NCHW int32 <-> z / z_hat NHWC */
int tmae_eb_symbols(const float* z, const tmae_eb_params* params, float* table, int n, int C, int HW, int* symbols,
                    void* stream);
int tmae_eb_dequantize(const int* symbols, const tmae_eb_params* params, float* table, int n, int C, int HW, void* zhat,
                       int zhat_dtype, void* stream);

/* inverse[b][perm[b][j]] = j (ids_shuffle from ids_restore for MCM.decompress) */
int tmae_invert_permutation(const int64_t* perm, int64_t* inverse, int n, int L, void* stream);

/* ---------------------------------------------------------------- entropy coding (host, no device work)
 * compressai 1.2.4's coder restated (csrc/rans.cpp; not vendored in the reference): 64-bit rANS, 16-bit
 * precision, bypass-escaped tails.  CDF tables are int32 [ncdf][cdf_stride] rows with cdf_sizes[c] valid
 * entries each (= _quantized_cdf / _cdf_length / _offset of an entropy model). */

/* compressai pmf_to_quantized_cdf (EntropyModel._pmf_to_cdf; update() at testing.py:223): cdf[n + 1] */
int tmae_pmf_to_quantized_cdf(const float* pmf, int n, int precision, int32_t* cdf);

/* BufferedRansEncoder (MCM.py:845): create, encode_with_indexes (882-887) any number of times, flush
 * (890; *nbytes = stream length), take the bytes, destroy. */
int tmae_rans_encoder_create(void** handle);
int tmae_rans_encode_with_indexes(void* handle, const int32_t* symbols, const int32_t* indexes, long long n,
                                  const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes,
                                  const int32_t* offsets, int ncdf);
int tmae_rans_encoder_flush(void* handle, long long* nbytes);
int tmae_rans_encoder_take(void* handle, uint8_t* out, long long cap);
int tmae_rans_encoder_destroy(void* handle);

/* RansDecoder (MCM.py:917-918): set_stream = create (the bytes are copied), decode_stream (941-943) any
 * number of times, each consuming the next n symbols, destroy. */
int tmae_rans_decoder_create(const uint8_t* data, long long len, void** handle);
int tmae_rans_decode_with_indexes(void* handle, const int32_t* indexes, long long n, const int32_t* cdfs,
                                  int cdf_stride, const int32_t* cdf_sizes, const int32_t* offsets, int ncdf,
                                  int32_t* out);
int tmae_rans_decoder_destroy(void* handle);

/* ---------------------------------------------------------------- Kodak eval harness (testing.py, §8f row 4)
 * HuffmanCoding (utils/huffman.py:6-171, host, no device work): the code table of a tensor of int64 values
 * (first-occurrence order, CPython heapq tie order, pre-order codes MSB-first in the low `lens` bits of
 * `codes`), its '0'/'1' encoding (out = NULL: only *nbits) and the prefix decode. */
int tmae_huffman_build(const int64_t* values, long long n, int64_t* syms, int32_t* lens, uint64_t* codes, int cap,
                       int* nsym);
int tmae_huffman_encode(const int64_t* values, long long n, const int64_t* syms, const int32_t* lens,
                        const uint64_t* codes, int nsym, char* out, long long cap, long long* nbits);
int tmae_huffman_decode(const char* bits, long long nbits, const int64_t* syms, const int32_t* lens,
                        const uint64_t* codes, int nsym, int64_t* out, long long cap, long long* nout);

/* compute_metrics (testing.py:40-49) on f32 NCHW images in [0, 1]: both rounded to 0..255, then
 * out[0] = PSNR over the batch (max 255), out[1] = pytorch_msssim.ms_ssim(data_range=255) (device). */
long long tmae_metrics_workspace(int n, int C, int H, int W); /* floats */
int tmae_image_metrics(const float* org, const float* rec, int n, int C, int H, int W, float* work, long long work_elems,
                       float* out, void* stream);

/* patch importance scores, the total_scores input of MCM.forward (generate_scores_file.py:19-31, utils/map.py,
 * utils/distribution.py; cv2 semantics as restated in oracle/scores_oracle.py): n grayscale uint8 images
 * [n][H][W] -> scores [n][(size/patch)^2] f32 (device, no host round trip). */
long long tmae_image_scores_workspace(int n, int H, int W, int size); /* bytes */
int tmae_image_scores(const unsigned char* gray, int n, int H, int W, int size, int patch, unsigned char* work,
                      long long work_bytes, float* scores, void* stream);

/* ---------------------------------------------------------------- VGG16 feature loss (MCM.forward_loss,
 * models/Compression/loss/vgg.py:86-115 with common/image_utils.py:4-23).  The convolutions are tmae_conv3x3
 * (act TMAE_ACT_RELU) and tmae_conv_dgrad; these are the glue kernels, NHWC, dtype = operand type. */
/* de_normalize + normalize_batch: x NCHW f32 [n][C<=3][H][W] -> y NHWC [n][H][W][CP] (channels >= C zero) */
int tmae_vgg_prep(const float* x, int n, int C, int H, int W, int CP, void* y, int dtype, void* stream);
/* its backward: g NHWC [n][H][W][CP] -> dx NCHW f32 [n][C][H][W] */
int tmae_vgg_prep_bwd(const void* g, int n, int C, int H, int W, int CP, float* dx, int dtype, void* stream);
/* 2x2 / stride 2 max pool (nn.MaxPool2d(2, 2)), argmax (0..3, first maximum) into arg when non-NULL */
int tmae_maxpool2(const void* x, int n, int H, int W, int C, void* y, unsigned char* arg, int dtype, void* stream);
/* dx [n][H][W][C] = scatter of dy to the argmax (+ add when non-NULL) */
int tmae_maxpool2_bwd(const void* dy, const unsigned char* arg, int n, int H, int W, int C, void* dx, const void* add,
                      int dtype, void* stream);
/* g *= (y > 0)  (ReLU backward from the ReLU output) */
int tmae_relu_mask(void* g, const void* y, long long n, int dtype, void* stream);
/* out[0] (accumulate ? += : =) mean((a - b)^2) (nn.MSELoss); part >= 1024 doubles */
int tmae_mse(const void* a, const void* b, long long n, double* part, float* out, int accumulate, int dtype,
             void* stream);
/* da = g[0] * 2 (a - b) / n */
int tmae_mse_bwd(const void* a, const void* b, long long n, const float* g, void* da, int dtype, void* stream);

/* ================================================================ training (MCM.forward backward,
 * driven by utils/engine.py:75-91: loss.backward(), clip_grad_norm_, Adam, aux Adam)
 * Every gradient is f32; GEMM operands are in `dtype` like the forward. */

/* forward extras: tmae_linear_fwd + the pre-activation (GELU input) copy `pre` (dtype of y, ld ldp) */
int tmae_linear_fwd_pre(const void* x, int x_f32, int ldx, int row_group, int group_stride, int row_offset,
                        const void* w, const float* bias, void* y, int y_f32, int ldy, void* pre, int ldp, int M,
                        int N, int K, int act, int dtype, void* stream);
/* out = resid + x w^T + bias, out-of-place (autograd keeps the block input) */
int tmae_linear_residual_out(const void* x, int ldx, const void* w, const float* bias, const float* resid, float* out,
                             int ld, int M, int N, int K, int dtype, void* stream);
/* tmae_mha_fwd + the per-row log2-sum-exp lse[b][h][t] (base-2, of scores * scale * log2 e) */
int tmae_mha_fwd_lse(const void* qkv, void* out, float* lse, int B, int T, int H, int dh, float scale, int dtype,
                     void* stream);
/* timm Attention backward: dqkv [B*T][3*H*dh] (dtype) from qkv, o (forward output), dO, lse */
int tmae_mha_bwd(const void* qkv, const void* o, const void* dout, const float* lse, void* dqkv, int B, int T, int H,
                 int dh, float scale, int dtype, void* stream);
/* kept-patch im2col for the patch-embed weight gradient: out[n*keep][Kw] (dtype), Kw = C*P*P rounded up to a
 * multiple of 8 with a zero tail (patch 14: 588 -> 592) */
int tmae_patch_gather(const float* imgs, const int64_t* ids_shuffle, void* out, int n, int C, int H, int W, int patch,
                      int L, int keep, int dtype, void* stream);

/* weight gradient (split-K TN GEMM on the operands as the forward stored them):
 * out[m][n] = sum_k A(k, m) B(k, n); A dense (row k = source row (k/a_G)*a_Gs + a_off + k%a_G, lda);
 * B dense (same remap) or, b_conv = 1, the implicit im2col of a 3x3 conv (padding 1, stride b_stride) over
 * NHWC maps (channels [0, b_c1) from b, the rest from b2; column = tap * b_Cin + ci).  The split-K partials
 * ([splits][M][N] f32 in work, see tmae_wgrad_workspace) are summed in a fixed order and written to
 * out[o_base + m*o_sm + (n % o_cp)*o_sc + (n / o_cp)*o_st] (= or += with accumulate).
 * bias_out (optional): bias_out[m] (= or += with bias_accumulate) sum_k A(k, m), the bias gradient of the layer
 * whose output gradient A is (the reference's autograd column sum over rows), formed inside the same GEMM. */
typedef struct tmae_wgrad_args {
  const void* a; int lda; int a_G, a_Gs, a_off;
  const void* b; int ldb; int b_G, b_Gs, b_off;
  int b_conv; const void* b2; int b_c1, b_ld2, b_H, b_W, b_stride, b_Cin;
  int M, N, K;
  float* work; long long work_elems;
  float* out; long long o_base, o_sm, o_sc, o_st; int o_cp; int accumulate;
  float* bias_out; int bias_accumulate;
  int slot_div;  /* split-K sized for 1 / slot_div of the CU slots (0 or 1: the whole chip); a weight gradient on
                    a side stream shares the chip, and fewer splits write and reduce fewer partial slabs */
  /* nb > 1: nb problems of the same shape in one launch (the same layer of several slices' stacks), problem j's
   * a / b / b2 / out / bias_out at j * s_a / s_b / s_b2 / s_out / s_bias elements past the first's (work holds
   * nb problems' slabs: tmae_wgrad_workspace x nb) */
  int nb; long long s_a, s_b, s_b2, s_out, s_bias;
} tmae_wgrad_args;
int tmae_wgrad(const tmae_wgrad_args* args, int dtype, void* stream);
long long tmae_wgrad_workspace(int M, int N, int K, int dtype);
long long tmae_wgrad_workspace_nb(int M, int N, int K, int dtype, int slot_div, int nb);

/* data gradient of y = x w^T: dx[M][K] = dy[M][N] wt[K][N]^T (wt = w transposed, dtype); dy rows remapped
 * like tmae_linear_fwd.  out (dtype, or f32 with out_f32) = dx * gelu'(pre) when pre is given (the GELU
 * before this layer), acc32 (optional) += the same in f32. */
int tmae_dgrad_linear(const void* dy, int ldy, int row_group, int group_stride, int row_offset, const void* wt, int M,
                      int N, int K, void* out, int out_f32, int ldo, const void* pre, int ldp, float* acc32, int ld32,
                      int dtype, void* stream);

/* data gradient of a 3x3 conv (padding 1, stride 1 or 2) as a transposed-conv implicit GEMM:
 * dx [n*H*W][cin] from dy [n*Ho*Wo][cout] (dtype) and wd = weight as [cin][3][3][cout] (dtype).
 * Single output (out, dtype or f32, optionally * gelu'(pre)) or, acc[0] != NULL, routed f32 accumulation:
 * input channels [0, lim0) += into acc[0], [lim0, lim1) into acc[1], [lim1, cin) into acc[2]
 * (torch.cat inputs, MCM.py:761,766,780). */
typedef struct tmae_conv_dgrad_args {
  const void* dy; int ldy;
  int n, H, W, stride, cout, cin;
  const void* wd;
  void* out; int out_f32, ldo; const void* pre; int ldp;
  float* acc[3]; int ld_acc[3]; int lim[3];
  /* nb > 1: nb problems of the same shape (no routes), problem j at element offsets j * s_dy / s_wd / s_out / s_pre
     from the first's dy / wd / out / pre -- the mean and scale stacks of one slice (nb = 2), or of the batched
     slices 6..11 (nb = 12) as one launch (0 or 1: one problem) */
  int nb; long long s_dy, s_wd, s_out, s_pre;
} tmae_conv_dgrad_args;
int tmae_conv_dgrad(const tmae_conv_dgrad_args* args, int dtype, void* stream);

/* weight re-layout: dst (contiguous [d0][d1][d2][d3], dst_dtype) = src[i0*s0 + i1*s1 + i2*s2 + i3*s3] (f32) */
int tmae_relayout(const float* src, void* dst, int dst_dtype, int d0, int d1, int d2, int d3, long long s0, long long s1,
                  long long s2, long long s3, void* stream);
/* every relayout of a table in one launch: table[t] = {src, dst, dst_dtype | mode << 8, d1, d2, d3, s0, s1, s2, s3,
 * total, first_chunk} (int64, device memory), first_chunk = the chunks of the tensors before t (mode 0, a plain
 * or strided copy: ceil(total / 32768); mode 1, a 2-D transpose: 64 x 64 tiles (s1 != 0: also the plain cast of the
 * same [d3][total / d3] source into the address s1); mode 2, a per-row transpose:
 * rows; mode 3, a 3x3 conv weight [d1 = Cout][d2 = Cin][3][3] restricted to input channels [d3, d3 + s0) into
 * tmae_lic_stack's fragment order, total = 9 * ceil(s0 / 32) * ceil(Cout / 16) * 512; mode 4, the transposed,
 * tap-flipped weight of [d1 = Cout][d2 = Cin][3][3] (input Cout, output Cin) in the same order, total = 9 *
 * ceil(Cout / 32) * ceil(Cin / 16) * 512; modes 3 and 4: ceil(total / 72 / 256) chunks, 256 units of 9 taps x 8
 * elements each), then nchunks more int64: the row t of every chunk (ntensors * 12 + nchunks values in all) */
int tmae_relayout_multi(const long long* table, int ntensors, long long nchunks, void* stream);

/* bias gradient: out[c] (=/+=) sum over rows r of x[(r/G)*Gs + off + r%G][c]; work >= 256*C floats */
int tmae_colsum(const void* x, int x_dtype, int ld, int rows, int C, int row_group, int group_stride, int row_offset,
                float* work, long long work_elems, float* out, int accumulate, void* stream);

/* LayerNorm backward (x rows remapped as in the forward, dy dense f32): dx32[sr] = dres[sr] (optional) + dx,
 * dxop (optional, op_dtype) = the same; dgamma / dbeta (=/+=).  work >= 2*D*(rows/8 + 4) floats. */
int tmae_layernorm_bwd(const float* x, const float* gamma, const float* dy, const float* dres, float* dx32, void* dxop,
                       int op_dtype, int rows, int D, int row_group, int group_stride, int row_offset, float eps,
                       float* work, long long work_elems, float* dgamma, float* dbeta, float* dres_colsum, int accumulate,
                       void* stream);

/* subpel_conv3x3 (PixelShuffle(2)) backward: dpre [n*H*W][C4] = unshuffle(dy) * gelu'(pre) (pre optional) */
int tmae_unshuffle_bwd(const void* dy, int dy_f32, int ldy, const void* pre, int ldp, void* out, int n, int H, int W,
                       int C4, int dtype, void* stream);
/* out = dy * gelu'(pre), elementwise */
int tmae_gelu_bwd(const void* dy, int dy_f32, const void* pre, void* out, long long total, int dtype, void* stream);
/* y_hat = y_hat_pre + 0.5 tanh(t) (MCM.py:782-783): g = (g32 + g32b) (f32) + g16 (dtype), each optional;
 * dt = g * 0.5 (1 - tanh^2 t) (dtype), gsum = g (f32, optional) */
int tmae_lrp_bwd(const float* g32, int ld32, const float* g32b, int ld32b, const void* g16, int ld16, const float* t,
                 int ldt, void* dt, int lddt, float* gsum, int ldgs, int rows, int C, int dtype, void* stream);
/* strided 2-D copy, element size esz (2 or 4 bytes) */
int tmae_copy2d(const void* src, int lds, void* dst, int ldd, int rows, int cols, int esz, void* stream);
/* GaussianConditional likelihood + quantize_ste backward for one slice (MCM.py:767-776) */
int tmae_gc_bwd(const float* y, int ldy, int yoff, const float* mu, const float* sigma, int ld_ms, const float* noise,
                int Mtot, const float* glik, const float* gyp, int ldg, float* dy, int lddy, void* dmu, void* dsigma,
                int ldd, int n, int HW, int sw, int dtype, void* stream);
/* EntropyBottleneck likelihood backward (MCM.py:741-744): dz NHWC (= gzhat pass-through + likelihood path) and
 * every density parameter's gradient into `grads` (same struct, f32 gradient buffers; =/+=) */
int tmae_eb_bwd(const tmae_eb_params* params, const float* z, const float* noise, const float* glik,
                const float* gzhat, float* dz, int n, int C, int HW, const tmae_eb_params* grads, int accumulate,
                void* stream);
/* aux_loss backward w.r.t. quantiles (utils/engine.py:87) */
int tmae_eb_aux_bwd(const tmae_eb_params* params, const float* target, const float* gout, float* dquantiles, int C,
                    int accumulate, void* stream);
/* rate backward (rd_loss.py:19-20): dlik = gout[0] / (lik * -ln2 * num_pixels) */
int tmae_bpp_bwd(const float* lik, const float* gout, float* dlik, long long n, double num_pixels, void* stream);
/* patchify of the reconstruction gradient: out [n*L][P*P*C] (dtype) */
int tmae_patchify(const float* imgs, void* out, int n, int C, int H, int W, int patch, int dtype, void* stream);
/* decoder_embed backward: gather the kept tokens' rows of the decoder gradient (off-by-one cls, MCM.py:664-672)
 * into tok_grad [n*ntok][D] (dtype) and the mask_token gradient (mask_part >= n*D floats) */
int tmae_decoder_embed_bwd_gather(const float* dec_grad, const int64_t* ids_shuffle, void* tok_grad, int n, int ntok,
                                  int L, int D, int dtype, float* mask_part, float* dmask, int accumulate,
                                  void* stream);
/* out = a + b (f32) */
int tmae_add(const float* a, const float* b, float* out, long long n, void* stream);

/* optimizer over flat f32 buffers: torch.optim.Adam step `step` (1-based), gradients scaled by clip[0]
 * when clip != NULL */
int tmae_adam(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2, float eps,
              float weight_decay, int step, const float* clip, void* stream);
/* the same over many tensors: table (device int64) = ntensors x {p, g, m, v, n, first_chunk, step, bc}, then
 * nchunks more int64 (the row of every chunk); chunks of 1024 elements, nchunks in total; step = device address of
 * the tensor's int32 step count (torch.optim.Adam's per-parameter state["step"]), advanced by one before the
 * update on the stream, so a captured graph replays correct bias corrections; bc = device address of 2 f32 the
 * launch writes the tensor's bias corrections to (1 - b1^step, sqrt(1 - b2^step)) */
int tmae_adam_multi(const long long* table, int ntensors, long long nchunks, float lr, float beta1, float beta2,
                    float eps, float weight_decay, const float* clip, void* stream);
/* clip_grad_norm_: out[0] = ||g||_2, out[1] = min(1, max_norm / (norm + 1e-6)); work >= 2048 doubles */
int tmae_grad_norm(const float* g, long long n, double* work, float max_norm, float* out, void* stream);
/* g *= scale[0] */
int tmae_scale(float* g, long long n, const float* scale, void* stream);

/* ---------------------------------------------------------------- distortion (MCM.forward_loss, MCM.py:690-712)
 * SSIM (pytorch_msssim: 11-tap gaussian, sigma 1.5, valid filtering, K = (0.01, 0.03), data range 1) and L1
 * over P = N*C planes of H x W (f32 NCHW, H, W >= 11): out[0] = 1 - SSIM, out[1] = mean |x - y|.
 * hwork >= 5*P*H*(W-10) floats, dmaps (3*P*(H-10)*(W-10) floats; NULL when no backward follows),
 * part >= 2048 doubles.  Backward: gx = d(g0 * out[0] + g1 * out[1]) / dx with gout = {g0, g1} on the device,
 * vwork >= 3*P*H*(W-10) floats. */
int tmae_distortion_fwd(const float* x, const float* y, int P, int H, int W, float* hwork, float* dmaps, double* part,
                        float* out, void* stream);
int tmae_distortion_bwd(const float* x, const float* y, int P, int H, int W, const float* dmaps, float* vwork,
                        const float* gout, float* gx, void* stream);

/* diagnostics (no device work): writes into out[len] the name of the MFMA GEMM variant that
 * tmae_linear_fwd / tmae_conv3x3 launch for an M x N x K problem batched `batch` times (tile shape,
 * waves per workgroup, LDS ring), e.g. "ring<bf16,256x256,8w,BK32x4>". */
int tmae_gemm_plan(int M, int N, int K, int batch, int dtype, char* out, int len);

#ifdef __cplusplus
}
#endif

#endif /* TMAE_H */
