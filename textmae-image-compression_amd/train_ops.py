"""Tensor-level wrappers over the training entry points of the C ABI (include/tmae.h, "training").

Same conventions as ops.py: host-side checks, then one enqueue on torch's current stream; the
library never allocates, so workspaces come from a per-device scratch buffer that only grows.
Pointer arguments accept tensors or raw device addresses (offset views into a buffer).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import ConvDgradArgs, WgradArgs
from .ops import _p, _stream, dtype_code

_SCRATCH: dict = {}


def scratch(device, elems: int, slot: int = 0) -> torch.Tensor:
    """f32 workspace of at least `elems` elements (stream-ordered reuse; never freed while in use)"""
    key = (device, slot)
    t = _SCRATCH.get(key)
    if t is None or t.numel() < elems:
        t = torch.empty(max(int(elems), 1 << 16), dtype=torch.float32, device=device)
        _SCRATCH[key] = t
    return t


def _esz(t):
    return t.element_size()


# ------------------------------------------------------------------------------------- forward extras
def linear_pre(x, w, b, dtype, act, out, pre, M=None, ldx=None, row_group=None, group_stride=0, row_offset=0):
    """out = act(x W^T + b) and pre = x W^T + b (the GELU input kept for the backward)"""
    N, K = w.shape
    M = x.numel() // x.shape[-1] if M is None else M
    ldx = x.shape[-1] if ldx is None else ldx
    _lib.call("tmae_linear_fwd_pre", x.data_ptr(), int(x.dtype == torch.float32), ldx, row_group or M, group_stride,
              row_offset, w.data_ptr(), _p(b), out.data_ptr(), int(out.dtype == torch.float32), out.shape[-1],
              _p(pre), 0 if pre is None else pre.shape[-1], M, N, K, act, dtype_code(dtype), _stream())
    return out


def linear_residual_out(x, w, b, resid, out, dtype):
    N, K = w.shape
    M = x.numel() // K
    _lib.call("tmae_linear_residual_out", x.data_ptr(), K, w.data_ptr(), _p(b), resid.data_ptr(), out.data_ptr(),
              out.shape[-1], M, N, K, dtype_code(dtype), _stream())
    return out


def mha_lse(qkv, B, T, H, dh, scale, dtype, out, lse):
    _lib.call("tmae_mha_fwd_lse", qkv.data_ptr(), out.data_ptr(), lse.data_ptr(), B, T, H, dh, float(scale),
              dtype_code(dtype), _stream())
    return out


def mha_bwd(qkv, o, dout, lse, dqkv, B, T, H, dh, scale, dtype):
    _lib.call("tmae_mha_bwd", qkv.data_ptr(), o.data_ptr(), dout.data_ptr(), lse.data_ptr(), dqkv.data_ptr(), B, T, H,
              dh, float(scale), dtype_code(dtype), _stream())
    return dqkv


def patch_gather(imgs, ids, out, keep, patch, dtype):
    n, C, H, W = imgs.shape
    L = ids.shape[1]
    _lib.call("tmae_patch_gather", imgs.data_ptr(), ids.data_ptr(), out.data_ptr(), n, C, H, W, patch, L, keep,
              dtype_code(dtype), _stream())
    return out


# ------------------------------------------------------------------------------------- gradients
def wgrad(a, b, M, N, K, out, dtype, lda=None, ldb=None, a_remap=(None, 0, 0), b_remap=(None, 0, 0), conv=None,
          layout="dense", cin_total=None, ci_off=0, accumulate=False, bias=None, bias_accumulate=False, ws_slot=1,
          slot_div=1, batch=None):
    """out <- sum_k A(k, m) B(k, n) in the parameter's layout; bias (optional) <- sum_k A(k, m), the bias
    gradient of the layer whose output gradient A is, formed by the same GEMM.
    layout: "dense" (out [M][N]), "dense_t" (out [N][M]: ConvTranspose2d 1x1 weights), "conv"
    (out [M][cin_total][3][3], columns of B = tap * Cin + ci land at input channel ci_off + ci).
    conv = dict(x2=None, c1=..., ld2=0, H=, W=, stride=, cin=) selects the implicit im2col of B.
    batch = (nb, s_a, s_b, s_b2, s_out, s_bias): nb problems of this shape in one launch, problem j's operands /
    outputs j * s elements past the first's (the same layer of several slices' stacks)."""
    dev = out.device
    code = dtype_code(dtype)
    nb = batch[0] if batch is not None else 1
    need = _lib.value("tmae_wgrad_workspace_nb", M, N, K, code, int(slot_div), nb)
    ws = scratch(dev, need, slot=ws_slot)  # slot 4: the side stream's weight gradients (mcm_train._wg)
    args = WgradArgs()
    args.a, args.lda = _p(a), (lda if lda is not None else M)
    G, Gs, off = a_remap
    args.a_G, args.a_Gs, args.a_off = (G or (1 << 30)), Gs, off
    args.b = _p(b)
    G, Gs, off = b_remap
    args.b_G, args.b_Gs, args.b_off = (G or (1 << 30)), Gs, off
    if conv is not None:
        args.b_conv = 1
        args.b2 = _p(conv.get("x2"))
        args.b_c1 = conv["c1"]
        args.ldb = ldb if ldb is not None else conv["c1"]
        args.b_ld2 = conv.get("ld2", 0)
        args.b_H, args.b_W, args.b_stride, args.b_Cin = conv["H"], conv["W"], conv.get("stride", 1), conv["cin"]
    else:
        args.ldb = ldb if ldb is not None else N
    args.M, args.N, args.K = M, N, K
    args.work, args.work_elems = ws.data_ptr(), ws.numel()
    args.out = out.data_ptr()
    if layout == "dense":
        args.o_base, args.o_sm, args.o_sc, args.o_st, args.o_cp = 0, N, 1, 0, N
    elif layout == "dense_t":
        args.o_base, args.o_sm, args.o_sc, args.o_st, args.o_cp = 0, 1, M, 0, N
    elif layout == "conv":
        cin = conv["cin"]
        ct = cin_total if cin_total is not None else cin
        args.o_base, args.o_sm, args.o_sc, args.o_st, args.o_cp = ci_off * 9, ct * 9, 9, 1, cin
    else:
        raise ValueError(layout)
    args.accumulate = int(accumulate)
    args.bias_out = _p(bias)
    args.bias_accumulate = int(bias_accumulate)
    args.slot_div = int(slot_div)
    if batch is not None:
        args.nb, args.s_a, args.s_b, args.s_b2, args.s_out, args.s_bias = batch
    _lib.call("tmae_wgrad", ctypes.byref(args), code, _stream())
    return out


def dgrad_linear(dy, wt, M, N, K, dtype, out=None, pre=None, acc32=None, ldy=None, row_group=None, group_stride=0,
                 row_offset=0, ldo=None):
    """dx[M][K] = dy[M][N] W (wt = W^T [K][N] in dtype); out (dtype or f32) = dx * gelu'(pre); acc32 += dx"""
    _lib.call("tmae_dgrad_linear", _p(dy), ldy if ldy is not None else N, row_group or M, group_stride, row_offset,
              _p(wt), M, N, K, _p(out), int(out is not None and out.dtype == torch.float32),
              ldo if ldo is not None else K, _p(pre), K if pre is None else pre.shape[-1], _p(acc32),
              K if acc32 is None else acc32.shape[-1], dtype_code(dtype), _stream())


def conv_dgrad(dy, wd, n, H, W, stride, cout, cin, dtype, out=None, pre=None, ldy=None, ldo=None, ldp=None,
               routes=None, out_f32=None, second=None, batch=None):
    """dx [n*H*W][cin] of a 3x3 conv from dy [n*Ho*Wo][cout]; wd = weight as [cin][3][3][cout] (dtype).
    routes: [(acc_f32, ld, ncols), ...] (<= 3, f32 +=, consecutive input-channel ranges).
    second = (dy2, wd2, out2, pre2): a second problem of the same shape and layout in the same launch (no routes).
    batch = (nb, s_dy, s_wd, s_out, s_pre): nb problems, problem j's dy / wd / out / pre j * s elements past the
    first's (no routes)"""
    a = ConvDgradArgs()
    if batch is not None:
        a.nb, a.s_dy, a.s_wd, a.s_out, a.s_pre = batch
    if second is not None:
        def off(t2, t1, what):
            if t2.dtype != t1.dtype:
                raise ValueError(f"conv_dgrad second problem: {what} dtype {t2.dtype} != {t1.dtype}")
            d = t2.data_ptr() - t1.data_ptr()
            if d % t1.element_size():
                raise ValueError(f"conv_dgrad second problem: {what} offset {d} B is not whole elements")
            return d // t1.element_size()
        dy2, wd2, out2, pre2 = second
        a.nb = 2
        a.s_dy, a.s_wd, a.s_out = off(dy2, dy, "dy"), off(wd2, wd, "wd"), off(out2, out, "out")
        if (pre is None) != (pre2 is None):
            raise ValueError("conv_dgrad second problem: pre given for one problem only")
        a.s_pre = off(pre2, pre, "pre") if pre is not None else 0
    a.dy, a.ldy = _p(dy), ldy if ldy is not None else cout
    a.n, a.H, a.W, a.stride, a.cout, a.cin = n, H, W, stride, cout, cin
    a.wd = _p(wd)
    if routes:
        lim = 0
        for i in range(3):
            if i < len(routes):
                acc, ld, nc = routes[i]
                a.acc[i] = _p(acc)
                a.ld_acc[i] = ld
                lim += nc
            a.lim[i] = lim
        if lim != cin:
            raise ValueError(f"conv_dgrad routes cover {lim} of {cin} channels")
    else:
        a.out = _p(out)
        a.out_f32 = int(out_f32 if out_f32 is not None else (isinstance(out, torch.Tensor) and out.dtype == torch.float32))
        a.ldo = ldo if ldo is not None else cin
        a.pre = _p(pre)
        a.ldp = ldp if ldp is not None else cin
    _lib.call("tmae_conv_dgrad", ctypes.byref(a), dtype_code(dtype), _stream())


def relayout(src, dst, dims, strides):
    """dst (contiguous dims) = cast(src[sum i_k * s_k]); up to 4 dims"""
    dims = list(dims) + [1] * (4 - len(dims))
    strides = list(strides) + [0] * (4 - len(strides))
    _lib.call("tmae_relayout", _p(src), _p(dst), dtype_code(dst.dtype), *dims, *strides, _stream())
    return dst


def colsum(x, rows, C, out, ld=None, row_group=None, group_stride=0, row_offset=0, accumulate=False, x_dtype=None):
    dev = out.device
    ws = scratch(dev, 256 * C, slot=2)
    xd = x_dtype if x_dtype is not None else x.dtype
    _lib.call("tmae_colsum", _p(x), dtype_code(xd), ld if ld is not None else C, rows, C, row_group or max(rows, 1),
              group_stride, row_offset, ws.data_ptr(), ws.numel(), out.data_ptr(), int(accumulate), _stream())
    return out


def layernorm_bwd(x, gamma, dy, dx32, rows, D, eps, dgamma, dbeta, dres=None, dxop=None, row_group=None,
                  group_stride=0, row_offset=0, accumulate=False, dres_colsum=None):
    """LayerNorm backward; dres_colsum (optional) receives the column sums of dres over the same rows
    (the bias gradient of the Linear whose output the residual adds), folded with dgamma / dbeta"""
    ws = scratch(dx32.device, 3 * D * (rows // 8 + 8), slot=2)
    op = dxop.dtype if dxop is not None else torch.float32
    _lib.call("tmae_layernorm_bwd", _p(x), _p(gamma), _p(dy), _p(dres), _p(dx32), _p(dxop), dtype_code(op), rows, D,
              row_group or max(rows, 1), group_stride, row_offset, float(eps), ws.data_ptr(), ws.numel(),
              _p(dgamma), _p(dbeta), _p(dres_colsum), int(accumulate), _stream())


def unshuffle_bwd(dy, ldy, pre, ldp, out, n, H, W, C4, dtype, dy_f32):
    _lib.call("tmae_unshuffle_bwd", _p(dy), int(dy_f32), ldy, _p(pre), ldp, _p(out), n, H, W, C4, dtype_code(dtype),
              _stream())


def lrp_bwd(t, ldt, dt, lddt, rows, C, dtype, g32=None, ld32=0, g16=None, ld16=0, gsum=None, ldgs=0, g32b=None,
            ld32b=0):
    _lib.call("tmae_lrp_bwd", _p(g32), ld32, _p(g32b), ld32b, _p(g16), ld16, _p(t), ldt, _p(dt), lddt, _p(gsum), ldgs,
              rows, C, dtype_code(dtype), _stream())


def gc_bwd(y, ldy, yoff, mu, sigma, ld_ms, noise, Mtot, glik, gyp, ldg, dy, lddy, dmu, dsigma, ldd, n, HW, sw, dtype):
    _lib.call("tmae_gc_bwd", _p(y), ldy, yoff, _p(mu), _p(sigma), ld_ms, _p(noise), Mtot, _p(glik), _p(gyp), ldg,
              _p(dy), lddy, _p(dmu), _p(dsigma), ldd, n, HW, sw, dtype_code(dtype), _stream())


def eb_bwd(params, z, noise, glik, gzhat, dz, n, C, HW, grads, accumulate=False):
    _lib.call("tmae_eb_bwd", ctypes.byref(params), _p(z), _p(noise), _p(glik), _p(gzhat), _p(dz), n, C, HW,
              ctypes.byref(grads), int(accumulate), _stream())


def eb_aux_bwd(params, target, gout, dq, C, accumulate=False):
    _lib.call("tmae_eb_aux_bwd", ctypes.byref(params), _p(target), _p(gout), _p(dq), C, int(accumulate), _stream())


def bpp_bwd(lik, gout, dlik, num_pixels):
    _lib.call("tmae_bpp_bwd", _p(lik), _p(gout), _p(dlik), lik.numel(), float(num_pixels), _stream())
    return dlik


def mae_loss_bwd(pred, imgs, ids_restore, keep, patch, norm_pix, dloss, dpred, out, dtype):
    """models_mae.forward_loss backward -> out [n*L, p*p*C] in `dtype` (dloss 1-element f32 or None; dpred the
    incoming gradient of pred itself, f32, or None)"""
    n, C, H, W = imgs.shape
    _lib.call("tmae_mae_loss_bwd", pred.data_ptr(), imgs.data_ptr(), ids_restore.data_ptr(), n, C, H, W, patch, keep,
              int(bool(norm_pix)), _p(dloss), _p(dpred), out.data_ptr(), dtype_code(dtype), _stream())
    return out


def patchify(imgs, out, patch, dtype):
    n, C, H, W = imgs.shape
    _lib.call("tmae_patchify", imgs.data_ptr(), out.data_ptr(), n, C, H, W, patch, dtype_code(dtype), _stream())
    return out


def decoder_embed_bwd_gather(dec_grad, ids, tok_grad, n, ntok, L, D, dtype, dmask=None, accumulate=False):
    part = scratch(dec_grad.device, n * D, slot=2) if dmask is not None else None
    _lib.call("tmae_decoder_embed_bwd_gather", dec_grad.data_ptr(), ids.data_ptr(), tok_grad.data_ptr(), n, ntok, L, D,
              dtype_code(dtype), _p(part), _p(dmask), int(accumulate), _stream())


def add(a, b, out):
    _lib.call("tmae_add", a.data_ptr(), b.data_ptr(), out.data_ptr(), out.numel(), _stream())
    return out


def copy2d(src, lds, dst, ldd, rows, cols, esz):
    _lib.call("tmae_copy2d", _p(src), lds, _p(dst), ldd, rows, cols, esz, _stream())


def adam(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, clip=None):
    _lib.call("tmae_adam", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), float(lr), float(beta1),
              float(beta2), float(eps), float(weight_decay), int(step), _p(clip), _stream())


def grad_norm(g, max_norm, out):
    """out[0] = ||g||, out[1] = clip factor (device f32 [2])"""
    work = scratch(g.device, 4096, slot=3)  # 2048 f64 partials
    _lib.call("tmae_grad_norm", g.data_ptr(), g.numel(), work.data_ptr(), float(max_norm), out.data_ptr(), _stream())
    return out


def scale_(g, factor):
    _lib.call("tmae_scale", g.data_ptr(), g.numel(), _p(factor), _stream())
