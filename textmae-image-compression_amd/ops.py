"""Tensor-level wrappers over the C ABI (include/tmae.h).

Each wrapper checks device / dtype / contiguity on the host, then enqueues the HIP kernel on
torch's current stream.  They allocate outputs with torch (the caching allocator owns all memory,
the library never allocates) unless an `out=` buffer is passed.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import ACT_GELU, ACT_NONE, TMAE_BF16, TMAE_F32, ConvArgs, EBParams, LicStackArgs

__all__ = [
    "ids_shuffle", "layernorm", "linear", "linear_residual", "patch_embed", "cls_rows", "mha", "decoder_embed",
    "mask_rows", "decoder_pred", "conv3x3", "lic_stack", "pack_lic_stack_weight", "lic_stack_fits", "gc_slices", "eb_likelihood", "eb_aux_loss",
    "gc_likelihood", "nhwc_to_nchw", "bpp", "gemm_plan", "dtype_code", "gc_slices_code", "gc_indexes",
    "gc_dequantize", "gc_pmf", "eb_pmf", "eb_symbols", "eb_dequantize", "invert_permutation", "mae_masking",
    "mae_loss", "TMAE_F32", "TMAE_BF16", "ACT_NONE", "ACT_GELU",
]


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    """device address of a tensor, a raw int address (offset views into a workspace), or None"""
    if t is None or isinstance(t, int):
        return t
    return t.data_ptr()


def _need(t: torch.Tensor, dtype=None, name="tensor"):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return TMAE_F32
    if dt == torch.bfloat16:
        return TMAE_BF16
    raise ValueError(f"unsupported compute dtype {dt}")


def gemm_plan(M: int, N: int, K: int, dtype: torch.dtype, batch: int = 1) -> str:
    """name of the MFMA GEMM variant the library launches for this problem (no device work)"""
    buf = ctypes.create_string_buffer(96)
    _lib.call("tmae_gemm_plan", M, N, K, batch, dtype_code(dtype), buf, len(buf))
    return buf.value.decode()


# --------------------------------------------------------------------------------------- masking
def ids_shuffle(scores: torch.Tensor, keep: int, sum_lanes: int = 8):
    """MCM.get_ids_shuffle + argsort (MCM.py:364-423, 579-580) -> (ids_shuffle, ids_restore) int64."""
    s = _need(scores.float().contiguous(), name="total_scores")
    n, L = s.shape
    shuf = torch.empty((n, L), dtype=torch.int64, device=s.device)
    rest = torch.empty_like(shuf)
    _lib.call("tmae_ids_shuffle", s.data_ptr(), shuf.data_ptr(), rest.data_ptr(), n, L, keep, sum_lanes, _stream())
    return shuf, rest


# --------------------------------------------------------------------------------------- transformer
def layernorm(x, weight, bias, eps, out_dtype, rows=None, row_group=None, group_stride=0, row_offset=0, out=None):
    _need(x, torch.float32, "x")
    D = x.shape[-1]
    rows = x.numel() // D if rows is None else rows
    row_group = rows if row_group is None else row_group
    if out is None:
        out = torch.empty((rows, D), dtype=out_dtype, device=x.device)
    _lib.call("tmae_layernorm_fwd", x.data_ptr(), weight.data_ptr(), bias.data_ptr(), out.data_ptr(), rows, D,
              max(row_group, 1), group_stride, row_offset, float(eps), dtype_code(out.dtype), _stream())
    return out


def linear(x, w, b, dtype, act=ACT_NONE, out=None, out_dtype=None, M=None, ldx=None, row_group=None, group_stride=0,
           row_offset=0, out32=None):
    """y = act(x W^T + b); x f32 or `dtype`; W [N][K] in `dtype`."""
    N, K = w.shape
    M = x.numel() // x.shape[-1] if M is None else M
    ldx = x.shape[-1] if ldx is None else ldx
    out_dtype = out_dtype or dtype
    if out is None:
        out = torch.empty((M, N), dtype=out_dtype, device=x.device)
    code = dtype_code(dtype)
    x_f32 = int(x.dtype == torch.float32)
    if code == TMAE_BF16 and not x_f32 and x.dtype != torch.bfloat16:
        raise ValueError("x must be f32 or bf16")
    if code == TMAE_F32 and (x.dtype != torch.float32 or out.dtype != torch.float32):
        raise ValueError("f32 path needs f32 tensors")
    _lib.call("tmae_linear_fwd", x.data_ptr(), x_f32, ldx, row_group or M, group_stride, row_offset, w.data_ptr(),
              _p(b), out.data_ptr(), int(out.dtype == torch.float32), out.shape[-1], _p(out32),
              0 if out32 is None else out32.shape[-1], M, N, K, act, code, _stream())
    return out


def linear_residual(x, w, b, resid, dtype):
    N, K = w.shape
    M = x.numel() // K
    _lib.call("tmae_linear_residual_fwd", x.data_ptr(), K, w.data_ptr(), _p(b), resid.data_ptr(), resid.shape[-1], M,
              N, K, dtype_code(dtype), _stream())
    return resid


_PATCH_WORK: dict = {}


def patch_embed(imgs, ids_shuffle, w, b, pos, tokens, keep, patch, dtype, patches=None):
    """kept-patch embedding (+ pos) into tokens rows 1..keep of every image.  Patches whose rows are whole 16-B
    chunks (P % 8 == 0), and every patch size when `patches` is given, are gathered first (into `patches`
    [n*keep][Kw] of dtype -- the training forward keeps them for the weight gradient -- else a cached workspace;
    Kw = C*P*P rounded up to 8, zero tail) and projected by the LDS-DMA GEMM; otherwise (ViT-H's patch 14 at
    inference) they are gathered value by value inside the GEMM."""
    n, C, H, W = imgs.shape
    D = w.shape[0]
    L = ids_shuffle.shape[1]
    if w.dim() != 2 or w.shape[1] != -(-C * patch * patch // 8) * 8 or not w.is_contiguous():
        raise ValueError(f"patch_embed: weight {tuple(w.shape)} must be contiguous [D][C*P*P rounded up to 8]")
    Kw = w.shape[1]  # C*P*P rounded up to 8 (the gathered rows' zero tail: patch 14, 588 -> 592)
    if patch % 8 == 0 or patches is not None:
        if patches is None:
            key = (imgs.device, dtype, n * keep * Kw)
            patches = _PATCH_WORK.get(key)
            if patches is None:
                patches = _PATCH_WORK[key] = torch.empty((n * keep, Kw), dtype=dtype, device=imgs.device)
            _lib.call("tmae_patch_gather", _need(imgs, torch.float32, "imgs").data_ptr(), ids_shuffle.data_ptr(),
                      patches.data_ptr(), n, C, H, W, patch, L, keep, dtype_code(dtype), _stream())
        elif tuple(patches.shape) != (n * keep, Kw):
            raise ValueError(f"patch_embed: gathered patches {tuple(patches.shape)} must be [{n * keep}][{Kw}]")
        _lib.call("tmae_patch_embed_gathered", patches.data_ptr(), ids_shuffle.data_ptr(), w.data_ptr(), b.data_ptr(),
                  pos.data_ptr(), tokens.data_ptr(), n, Kw, D, L, keep, dtype_code(dtype), _stream())
        return tokens
    _lib.call("tmae_patch_embed_fwd", _need(imgs, torch.float32, "imgs").data_ptr(), ids_shuffle.data_ptr(),
              w.data_ptr(), b.data_ptr(), pos.data_ptr(), tokens.data_ptr(), n, C, H, W, patch, D, L, keep,
              dtype_code(dtype), _stream())
    return tokens


def cls_rows(tokens, cls, pos, n, rows_per_img, D):
    _lib.call("tmae_cls_rows", tokens.data_ptr(), cls.data_ptr(), pos.data_ptr(), n, rows_per_img, D, _stream())


def mha(qkv, B, T, H, dh, scale, dtype, out=None):
    if out is None:
        out = torch.empty((B * T, H * dh), dtype=dtype, device=qkv.device)
    _lib.call("tmae_mha_fwd", qkv.data_ptr(), out.data_ptr(), B, T, H, dh, float(scale), dtype_code(dtype), _stream())
    return out


_QKV_ATTN_OK = {}


def qkv_attn_supported(T, H, dh, dtype):
    """a fused qkv + attention kernel exists for this shape (bf16 only)"""
    if dtype != torch.bfloat16:
        return False
    key = (T, H, dh)
    if key not in _QKV_ATTN_OK:
        _QKV_ATTN_OK[key] = bool(_lib.value("tmae_qkv_attn_supported", T, H, dh))
    return _QKV_ATTN_OK[key]


def qkv_attn(x, w, b, B, T, H, dh, scale, dtype, out):
    """out = attention(x W_qkv^T + b_qkv) in one launch, Q / K / V kept on chip (tmae_qkv_attn_fwd)"""
    _lib.call("tmae_qkv_attn_fwd", x.data_ptr(), w.data_ptr(), b.data_ptr(), out.data_ptr(), B, T, H, dh, float(scale),
              dtype_code(dtype), _stream())
    return out


def decoder_embed(x, w, b, pos, ids_shuffle, out, n, ntok, L, dtype):
    D, Din = w.shape
    _lib.call("tmae_decoder_embed_fwd", x.data_ptr(), int(x.dtype == torch.float32), w.data_ptr(), b.data_ptr(),
              pos.data_ptr(), ids_shuffle.data_ptr(), out.data_ptr(), n, ntok, L, Din, D, dtype_code(dtype),
              _stream())


def mask_rows(out, mask_token, pos, ids_shuffle, n, L, ntok, D):
    _lib.call("tmae_mask_rows", out.data_ptr(), mask_token.data_ptr(), pos.data_ptr(), ids_shuffle.data_ptr(), n, L,
              ntok, D, _stream())


def decoder_pred(x, w, b, imgs, n, L, patch, dtype, channel_planar=False):
    """channel_planar: w / b rows already in (c, py, px) order (see pred_channel_planar_perm)"""
    N, Din = w.shape
    C, H, W = imgs.shape[1:]
    _lib.call("tmae_decoder_pred_cp_fwd" if channel_planar else "tmae_decoder_pred_fwd", x.data_ptr(), w.data_ptr(),
              b.data_ptr(), imgs.data_ptr(), n, L, Din, C, H, W, patch, dtype_code(dtype), _stream())


def pred_channel_planar_perm(patch, chans):
    """row permutation taking decoder_pred rows (py, px, c) (MCM.py:524-546 "nhwpqc") to (c, py, px)"""
    return torch.arange(patch * patch * chans).view(patch, patch, chans).permute(2, 0, 1).reshape(-1)


# --------------------------------------------------------------------------------------- LIC
def conv3x3(x1, c1, ld1, n, H, W, w, b, y, ldy, cout, dtype, stride=1, act=ACT_NONE, pixel_shuffle=False,
            x2=None, c2=0, ld2=0, y_f32=None, y32=None, ld32=0, addend=None, ld_add=0, lrp_src=None, ld_src=0,
            y2=None, ldy2=0, nb=(1, 1), strides=None, pre=None, ldp=0):
    """Batched 3x3 conv (tmae_conv3x3).  Pointer arguments: tensors or raw device addresses.
    `strides` maps operand name (x1, x2, w, b, y, y32, a, src, y2, pre) -> (s1, s2) element strides for the
    nb[0] x nb[1] problems.  `pre` (training): pre-activation copy in the output's dtype / layout (the last
    lrp conv: f32 pre-tanh rows ldp apart)."""
    a = ConvArgs()
    a.x1, a.c1, a.ld1 = _p(x1), c1, ld1
    a.x2, a.c2, a.ld2 = _p(x2), c2, ld2
    a.n, a.H, a.W, a.stride = n, H, W, stride
    a.w, a.bias = _p(w), _p(b)
    a.cout, a.act, a.pixel_shuffle = cout, act, int(pixel_shuffle)
    if dtype == torch.float32:
        y_f32 = True  # the f32 path writes f32 everywhere
    elif y_f32 is None:
        y_f32 = isinstance(y, torch.Tensor) and y.dtype == torch.float32
    a.y, a.y_f32, a.ldy = _p(y), int(y_f32), ldy
    a.y32, a.ld32 = _p(y32), ld32
    a.addend, a.ld_add = _p(addend), ld_add
    a.lrp_src, a.ld_src = _p(lrp_src), ld_src
    a.y2, a.ldy2 = _p(y2), ldy2
    a.pre, a.ldp = _p(pre), ldp
    a.nb1, a.nb2 = nb
    for name, (s1, s2) in (strides or {}).items():
        setattr(a, f"{name}_s1", s1)
        setattr(a, f"{name}_s2", s2)
    _lib.call("tmae_conv3x3", ctypes.byref(a), dtype_code(dtype), _stream())


LSTK_MAXC, LSTK_MAXPIX = 224, 144  # lic_stack.hip: widest resident activation, pixels per workgroup


def _pad(c, m):
    return (c + m - 1) // m * m


def lic_stack_fits(G, cin0, couts):
    """True when tmae_lic_stack takes a stack of this shape (grid G x G, layer-0 input cin0 channels,
    output channels per layer): bf16 operands, activations resident in one workgroup's LDS"""
    return (G * G <= LSTK_MAXPIX and cin0 % 8 == 0 and _pad(cin0, 32) <= LSTK_MAXC and 1 <= len(couts) <= 5
            and all(c % 8 == 0 for c in couts) and all(_pad(c, 32) <= LSTK_MAXC for c in couts[:-1]))


def pack_lic_stack_weight(w: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """Conv weight [Cout][Cin][3][3] -> tmae_lic_stack's MFMA fragment order
    [tap 9][k-step Cin/32][cout fragment Cout/16][lane 64][8] (lane = 16 * k-group + cout row), zero-padded
    to multiples of 32 input / 16 output channels (flat, `dtype`)"""
    w = w.detach()
    co, ci = w.shape[:2]
    cip, cop = _pad(ci, 32), _pad(co, 16)
    t = torch.zeros(9, cop, cip, dtype=torch.float32, device=w.device)
    if ci:
        t[:, :co, :ci] = w.float().permute(2, 3, 0, 1).reshape(9, co, ci)
    nkc, nfr = cip // 32, cop // 16
    t = t.view(9, nfr, 16, nkc, 4, 8).permute(0, 3, 1, 4, 2, 5).contiguous()
    return t.view(-1).to(dtype)


def pack_lic_stack_weight_t(w: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """A 3x3 conv weight [Cout][Cin][3][3] as the weight of its transposed conv (the data gradient: input Cout
    channels, output Cin, taps flipped) in tmae_lic_stack's fragment order (relayout mode 4 builds the same)"""
    return pack_lic_stack_weight(w.detach().transpose(0, 1).flip(2, 3), dtype)


def lic_stack_bwd(n, G, dtop, ldt, c_top, weights, couts, pres, outs, nb=(1, 1), strides=None, routes=None):
    """The data-gradient chain of a slice stack's layers L-1..1 in one launch (tmae_lic_stack, TMAE_LIC_STACK_BWD):
    dtop [rows][c_top] (bf16, rows ldt apart) is the gradient of the stack's output; layer l (the transposed conv
    of forward layer L-1-l, weights[l] from pack_lic_stack_weight_t) writes outs[l] = (its conv) * GELU'(pres[l]),
    bf16 [rows][couts[l]].  `strides` maps x1, w<l>, s<l> (pres[l] / outs[l]) -> per-problem (s1, s2).
    routes (optional, one list per problem of (acc_f32, ld, ncols), <= 3 consecutive channel ranges): the last
    layer is the stack's first conv's input gradient, added into those accumulators (no pres / outs entry)."""
    a = LicStackArgs()
    if routes is not None:
        if nb[1] != 1:
            # the kernel steps routed accumulators by problem index along nb1 only
            raise ValueError("lic_stack_bwd routes: nb2 must be 1")
        if len(routes) > 1 and len(routes) != nb[0]:
            raise ValueError("lic_stack_bwd routes: one route list per problem")
        lim = 0
        for r in range(3):
            if r < len(routes[0]):
                acc, ld, nc = routes[0][r]
                a.racc[r], a.rld[r] = _p(acc), ld
                if len(routes) > 1 and nc:
                    steps = [_p(routes[k + 1][r][0]) - _p(routes[k][r][0]) for k in range(len(routes) - 1)]
                    if len(set(steps)) != 1 or steps[0] % 4:
                        raise ValueError("lic_stack_bwd routes: accumulators not at a constant stride")
                    a.rs[r] = steps[0] // 4  # problem k's accumulator = problem 0's + k * stride (f32 elements)
                lim += nc
            a.rlim[r] = lim
    a.n, a.G, a.nlayers = n, G, len(couts)
    a.nb1, a.nb2 = nb
    a.x1, a.c1, a.ld1 = _p(dtop), c_top, ldt
    a.flags = 2
    for l, (w, c) in enumerate(zip(weights, couts)):
        a.w[l], a.cout[l] = _p(w), c
        if l < len(pres):
            a.sv_pre[l], a.sv_act[l] = _p(pres[l]), _p(outs[l])
    for name, (s1, s2) in (strides or {}).items():
        if name[0] == "w":
            a.w_s[int(name[1:])][:] = (s1, s2)
        elif name[0] == "s":
            a.sv_s[int(name[1:])][:] = (s1, s2)
        else:
            getattr(a, f"{name}_s")[:] = (s1, s2)
    _lib.call("tmae_lic_stack", ctypes.byref(a), _stream())


def lic_latent_fits(G, cin):
    """True when tmae_lic_latent takes the latent partial sums of this shape (bf16, cin a multiple of 32)"""
    return G * G <= LSTK_MAXPIX and cin % 32 == 0 and 32 <= cin <= 384


def lic_latent(n, G, xs, ldx, cin, w, nfr, blk, f_off, f_lo, f_hi, y, ldy, y_s=None, biases=None, act=ACT_NONE,
               y_bf16=False):
    """Stride-1 3x3 conv with the input resident in LDS (tmae_lic_latent): for problem j, relative fragment r in
    [f_lo, f_hi): y + y_s[j] (elements), columns 16 r .. = act(bias_j + the conv of xs[j]'s channels [0, cin) with
    the packed weight fragments f_off[j] + r of w: blocks of nfr fragments blk elements apart (pack_lic_stack_weight,
    stacked)).  y_s defaults to 16 f_off[j] (the latent partial sums' column blocks).  Pointers: tensors or raw
    addresses."""
    a = _lib.LicLatentArgs()
    a.n, a.G, a.cin, a.nb = n, G, cin, len(xs)
    for j, (x, fo) in enumerate(zip(xs, f_off)):
        a.x[j] = _p(x)
        a.f_off[j] = fo
        a.y_s[j] = (16 * fo) if y_s is None else y_s[j]
        a.bias[j] = _p(biases[j]) if biases is not None else None
    a.ldx, a.w, a.nfr, a.blk = ldx, _p(w), nfr, blk
    a.f_lo, a.f_hi = f_lo, f_hi
    a.y, a.ldy = _p(y), ldy
    a.act, a.y_bf16 = act, int(y_bf16)
    _lib.call("tmae_lic_latent", ctypes.byref(a), _stream())


def lic_stack(n, G, x1, c1, ld1, weights, biases, couts, y, ldy, y_f32, x2=None, c2=0, ld2=0, addend=None, ld_add=0,
              lrp_src=None, ld_src=0, y2=None, ldy2=0, nb=(1, 1), strides=None, chain=None, save=None):
    """One slice-transform stack per (problem, image) (tmae_lic_stack).  weights: packed per layer
    (pack_lic_stack_weight, problems stacked); `strides` maps operand (x1, x2, w0..w4, b0..b4, a, y, src, y2)
    -> (s1, s2) element strides of the nb[0] x nb[1] problems.  Pointers: tensors or raw addresses.
    save (training): {"layers": [(pre, act, (s1, s2)) per non-last layer], "t": pre-tanh f32, "t_s": (s1, s2),
    "chain": [(pre, act, s) per lrp layer], "chain_t": ..., "chain_t_s": s} -- what the HIP backward reads."""
    a = LicStackArgs()
    a.n, a.G, a.nlayers = n, G, len(couts)
    a.nb1, a.nb2 = nb
    a.x1, a.c1, a.ld1 = _p(x1), c1, ld1
    a.x2, a.c2, a.ld2 = _p(x2), c2, ld2
    for l, (w, b, c) in enumerate(zip(weights, biases, couts)):
        a.w[l], a.bias[l], a.cout[l] = _p(w), _p(b), c
    a.addend, a.ld_add = _p(addend), ld_add
    a.y, a.y_f32, a.ldy = _p(y), int(y_f32), ldy
    a.lrp_src, a.ld_src = _p(lrp_src), ld_src
    a.y2, a.ldy2 = _p(y2), ldy2
    if chain is not None:  # the mean problem goes on with its slice's lrp stack (TMAE_LIC_STACK_CHAIN)
        a.flags = 1
        a.cn = len(chain["couts"])
        for l, (w, b, c) in enumerate(zip(chain["w"], chain["b"], chain["couts"])):
            a.cw[l], a.cb[l], a.ccout[l] = _p(w), _p(b), c
        a.cx1, a.cc1, a.cld1 = _p(chain["x1"]), chain["c1"], chain["ld1"]
        a.yv, a.ldyv = _p(chain["y"]), chain["ldy"]
        a.cadd, a.cld_add = _p(chain["add"]), chain["ld_add"]
        a.csrc, a.cld_src = _p(chain["ypre"]), chain["ld_ypre"]
        a.cy, a.cldy = _p(chain["out"]), chain["ld_out"]
        a.cy2, a.cldy2 = _p(chain.get("out2")), chain.get("ld_out2", 0)
        cs = chain.get("strides", {})  # per-slice (b2) element strides of the chain operands
        a.cs_x1, a.cs_yv, a.cs_src = cs.get("x1", 0), cs.get("y", 0), cs.get("ypre", 0)
        a.cs_add, a.cs_y, a.cs_y2 = cs.get("add", 0), cs.get("out", 0), cs.get("out2", 0)
        for l in range(a.cn):
            a.cs_w[l], a.cs_b[l] = cs.get(f"w{l}", 0), cs.get(f"b{l}", 0)
    for name, (s1, s2) in (strides or {}).items():
        if name[0] in "wb" and name[1:].isdigit():
            getattr(a, f"{name[0]}_s")[int(name[1:])][:] = (s1, s2)
        else:
            getattr(a, f"{name}_s")[:] = (s1, s2)
    if save is not None:  # training: per layer (pre, act, (s1, s2)) of the problems, and the lrp pre-tanh t
        for l, (pre, act, st) in enumerate(save.get("layers", [])):
            a.sv_pre[l], a.sv_act[l] = _p(pre), _p(act)
            a.sv_s[l][:] = st
        if save.get("t") is not None:
            a.sv_t = _p(save["t"])
            a.sv_t_s[:] = save.get("t_s", (0, 0))
        for l, (pre, act, st) in enumerate(save.get("chain", [])):
            a.csv_pre[l], a.csv_act[l] = _p(pre), _p(act)
            a.cs_sv[l] = st
        if save.get("chain_t") is not None:
            a.csv_t, a.cs_t = _p(save["chain_t"]), save.get("chain_t_s", 0)
    _lib.call("tmae_lic_stack", ctypes.byref(a), _stream())


def gc_slices(y, ldy, yoff, mu, sigma, ms_stride, ld_ms, noise, lik, Mtot, yhat, yhat_dtype, ld_yhat, yhat32, ld32, n,
              HW, nslices, sw):
    _lib.call("tmae_gc_slices_fwd", _p(y), ldy, yoff, _p(mu), _p(sigma), ms_stride, ld_ms, _p(noise), _p(lik), Mtot,
              _p(yhat), dtype_code(yhat_dtype), ld_yhat, _p(yhat32), ld32, n, HW, nslices, sw, _stream())


def mae_masking(noise: torch.Tensor, len_keep: int):
    """models_mae.random_masking indices: (ids_shuffle, ids_restore) int64 and the binary mask f32 [n, L]"""
    nz = _need(noise.float().contiguous(), name="noise")
    n, L = nz.shape
    shuf = torch.empty((n, L), dtype=torch.int64, device=nz.device)
    rest = torch.empty_like(shuf)
    mask = torch.empty((n, L), dtype=torch.float32, device=nz.device)
    _lib.call("tmae_mae_masking", nz.data_ptr(), shuf.data_ptr(), rest.data_ptr(), mask.data_ptr(), n, L, len_keep,
              _stream())
    return shuf, rest, mask


_MAE_WORK = {}


def mae_loss(pred, imgs, ids_restore, len_keep, patch, norm_pix_loss):
    """models_mae.forward_loss -> 0-d f32 device tensor"""
    p = _need(pred.contiguous(), torch.float32, "pred")
    x = _need(imgs.contiguous(), torch.float32, "imgs")
    n, C, H, W = x.shape
    work = _MAE_WORK.get(x.device)
    if work is None:
        work = _MAE_WORK[x.device] = torch.empty(1024, dtype=torch.float64, device=x.device)
    out = torch.empty((), dtype=torch.float32, device=x.device)
    _lib.call("tmae_mae_loss", p.data_ptr(), x.data_ptr(), _need(ids_restore, torch.int64, "ids_restore").data_ptr(),
              n, C, H, W, patch, len_keep, int(bool(norm_pix_loss)), work.data_ptr(), out.data_ptr(), _stream())
    return out


def gc_slices_code(y, ldy, yoff, mu, sigma, ms_stride, ld_ms, lik, Mtot, yhat, yhat_dtype, ld_yhat, yhat32, ld32, n,
                   HW, nslices, sw, symbols, indexes, scale_table):
    """eval slice step of MCM.compress: gc_slices outputs + int32 symbols / scale indexes in coder order"""
    st = _need(scale_table.contiguous(), torch.float32, "scale_table")
    _lib.call("tmae_gc_slices_code", _p(y), ldy, yoff, _p(mu), _p(sigma), ms_stride, ld_ms, _p(lik), Mtot, _p(yhat),
              dtype_code(yhat_dtype), ld_yhat, _p(yhat32), ld32, n, HW, nslices, sw, _p(symbols), _p(indexes),
              st.data_ptr(), st.numel(), _stream())


def gc_indexes(sigma, ms_stride, ld_ms, n, HW, nslices, sw, scale_table, scale_bound, indexes):
    st = _need(scale_table.contiguous(), torch.float32, "scale_table")
    _lib.call("tmae_gc_indexes", _p(sigma), ms_stride, ld_ms, n, HW, nslices, sw, st.data_ptr(), st.numel(),
              float(scale_bound), _p(indexes), _stream())


def gc_dequantize(symbols, mu, ms_stride, ld_ms, n, HW, nslices, sw, yoff, yhat, yhat_dtype, ld_yhat, yhat32, ld32):
    _lib.call("tmae_gc_dequantize", _p(symbols), _p(mu), ms_stride, ld_ms, n, HW, nslices, sw, yoff, _p(yhat),
              dtype_code(yhat_dtype), ld_yhat, _p(yhat32), ld32, _stream())


def gc_pmf(scale_table, pmf_center, max_length):
    """GaussianConditional.update pmf rows + tail masses (device tensors)"""
    st = _need(scale_table.contiguous(), torch.float32, "scale_table")
    c = _need(pmf_center.to(torch.int32).contiguous(), torch.int32, "pmf_center")
    pmf = torch.empty((st.numel(), max_length), dtype=torch.float32, device=st.device)
    tail = torch.empty(st.numel(), dtype=torch.float32, device=st.device)
    _lib.call("tmae_gc_pmf", st.data_ptr(), c.data_ptr(), st.numel(), max_length, pmf.data_ptr(), tail.data_ptr(),
              _stream())
    return pmf, tail


def eb_pmf(eb, pmf_start, max_length):
    """EntropyBottleneck.update pmf rows + tail masses (device tensors)"""
    C = eb.channels
    dev = eb.quantiles.device
    start = _need(pmf_start.float().contiguous(), torch.float32, "pmf_start")
    pmf = torch.empty((C, max_length), dtype=torch.float32, device=dev)
    tail = torch.empty(C, dtype=torch.float32, device=dev)
    table = torch.empty((C, 59), dtype=torch.float32, device=dev)
    params = _eb_params(eb)
    _lib.call("tmae_eb_pmf", params, table.data_ptr(), start.data_ptr(), C, max_length, pmf.data_ptr(),
              tail.data_ptr(), _stream())
    return pmf, tail


def eb_symbols(eb, z_nhwc, n, C, HW, out=None, table=None):
    """round(z - median) as int32 NCHW [n, C, HW] from NHWC z"""
    dev = z_nhwc.device
    out = torch.empty((n, C, HW), dtype=torch.int32, device=dev) if out is None else out
    table = torch.empty((C, 59), dtype=torch.float32, device=dev) if table is None else table
    params = _eb_params(eb)
    _lib.call("tmae_eb_symbols", z_nhwc.data_ptr(), params, table.data_ptr(), n, C, HW, _p(out), _stream())
    return out


def eb_dequantize(eb, symbols, n, C, HW, zhat, table=None):
    """z_hat (NHWC, zhat's dtype) = symbols (NCHW int32) + median"""
    dev = zhat.device
    table = torch.empty((C, 59), dtype=torch.float32, device=dev) if table is None else table
    params = _eb_params(eb)
    _lib.call("tmae_eb_dequantize", _p(symbols), params, table.data_ptr(), n, C, HW, _p(zhat), dtype_code(zhat.dtype),
              _stream())
    return zhat


def invert_permutation(perm):
    p = _need(perm.to(torch.int64).contiguous(), torch.int64, "permutation")
    n, L = p.shape
    inv = torch.empty_like(p)
    _lib.call("tmae_invert_permutation", p.data_ptr(), inv.data_ptr(), n, L, _stream())
    return inv


def _eb_params(eb) -> EBParams:
    p = EBParams()
    for i in range(5):
        p.matrix[i] = getattr(eb, f"_matrix{i}").data_ptr()
        p.bias[i] = getattr(eb, f"_bias{i}").data_ptr()
        if i < 4:
            p.factor[i] = getattr(eb, f"_factor{i}").data_ptr()
    p.quantiles = eb.quantiles.data_ptr()
    return p


def eb_likelihood(eb, z_nhwc, n, C, HW, noise=None, lik=None, zhat=None, table=None):
    """EntropyBottleneck forward on NHWC z: returns (lik NCHW, z_hat NHWC in zhat's dtype, default f32)."""
    dev = z_nhwc.device
    if lik is None:
        lik = torch.empty((n, C, HW), dtype=torch.float32, device=dev)
    if zhat is None:
        zhat = torch.empty((n * HW, C), dtype=torch.float32, device=dev)
    if table is None:
        table = torch.empty((C, 59), dtype=torch.float32, device=dev)
    params = _eb_params(eb)
    _lib.call("tmae_eb_likelihood_fwd", z_nhwc.data_ptr(), params, _p(noise), lik.data_ptr(), _p(zhat),
              dtype_code(zhat.dtype), table.data_ptr(), n, C, HW, _stream())
    return lik, zhat


def eb_aux_loss(eb, out=None, table=None):
    C = eb.channels
    dev = eb.quantiles.device
    out = torch.empty((), dtype=torch.float32, device=dev) if out is None else out
    table = torch.empty((C, 59), dtype=torch.float32, device=dev) if table is None else table
    params = _eb_params(eb)
    _lib.call("tmae_eb_aux_loss", params, eb.target.data_ptr(), out.data_ptr(), table.data_ptr(), C, _stream())
    return out


def gc_likelihood(x, scales, means=None, noise=None, scale_bound=0.11):
    x = _need(x.contiguous(), torch.float32, "inputs")
    lik = torch.empty_like(x)
    xt = torch.empty_like(x)
    _lib.call("tmae_gc_likelihood_fwd", x.data_ptr(), _need(scales.contiguous(), torch.float32, "scales").data_ptr(),
              _p(None if means is None else means.contiguous()), _p(noise), xt.data_ptr(), lik.data_ptr(), x.numel(),
              float(scale_bound), _stream())
    return xt, lik


def nhwc_to_nchw(x, ldx, n, C, H, W, out=None):
    out = torch.empty((n, C, H, W), dtype=torch.float32, device=x.device) if out is None else out
    _lib.call("tmae_nhwc_to_nchw", x.data_ptr(), ldx, out.data_ptr(), n, C, H * W, _stream())
    return out


def crop_normalize_u8(src, crops, size, mean, std, out=None):
    """random-crop loader sample: src uint8 [nsrc, H, W, 3] (device), crops int32 [B, 3] = (image, top, left)
    (device) -> (crop / 255 - mean) / std as f32 [B, 3, size, size] (utils/dataloader.py:58-61)"""
    import ctypes

    assert src.dtype == torch.uint8 and src.dim() == 4 and src.shape[3] == 3 and src.is_contiguous()
    crops = _need(crops.contiguous(), torch.int32, "crops")
    B = crops.shape[0]
    out = torch.empty((B, 3, size, size), dtype=torch.float32, device=src.device) if out is None else out
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    s = (ctypes.c_float * 3)(*[float(v) for v in std])
    _lib.call("tmae_crop_normalize_u8", src.data_ptr(), src.shape[0], src.shape[1], src.shape[2], crops.data_ptr(), B,
              size, m, s, out.data_ptr(), _stream())
    return out


_BPP_WORK = {}


def bpp(y_lik, z_lik, num_pixels):
    """sum(log y_lik) + sum(log z_lik), / (-ln 2 * num_pixels): a 0-d f32 device tensor (rd_loss.py:19-20)."""
    y = _need(y_lik.contiguous(), torch.float32, "y likelihood")
    z = _need(z_lik.contiguous(), torch.float32, "z likelihood")
    work = _BPP_WORK.get(y.device)
    if work is None:
        work = _BPP_WORK[y.device] = torch.empty(512, dtype=torch.float64, device=y.device)
    out = torch.empty((), dtype=torch.float32, device=y.device)
    _lib.call("tmae_bpp_sum", y.data_ptr(), y.numel(), z.data_ptr(), z.numel(), work.data_ptr(), out.data_ptr(),
              float(num_pixels), _stream())
    return out
