"""Training path on the MI355X: backward kernels vs torch autograd (fp32 CPU), and the whole
MCM.forward backward vs the autograd-faithful oracle (oracle/train_oracle.py).

Tolerances: f32 operand path max|a-b| / max|b| <= 1e-3 per tensor (bit-level GELU / erf approximations
and summation order); bf16 operand path relative L2 <= 3e-2 against the fp32 reference.
"""
import math
import os

import numpy as np
import pytest
import torch
from parity_log import check  # noqa: E402
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    den = b.abs().max().item()
    return (a - b).abs().max().item() / (den if den > 0 else 1.0)


def _rel2(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    den = b.norm().item()
    return (a - b).norm().item() / (den if den > 0 else 1.0)


@pytest.fixture(scope="module")
def T():
    import textmae_amd  # noqa: F401
    from textmae_amd import train_ops

    return train_ops


def _rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


# ------------------------------------------------------------------------------ wgrad (TN GEMM)
@pytest.mark.parametrize("K,M,N", [(300, 256, 136), (1000, 72, 200), (9280, 768, 3072), (16448, 1536, 512)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_wgrad_dense(T, K, M, N, dt):
    if dt == torch.float32 and K * M * N > 3e9:
        pytest.skip("f32 parity path checked on the smaller shapes")
    a, b = _rnd(K, M, seed=1), _rnd(K, N, seed=2)
    ref = (a.to(dt).double().t() @ b.to(dt).double()).float()
    out = torch.empty(M, N, device="cuda")
    T.wgrad(a.cuda().to(dt), b.cuda().to(dt), M, N, K, out, dt)
    torch.cuda.synchronize()
    check("_rel:out", _rel(out, ref), (1e-5 if dt == torch.float32 else 2e-3))


def test_wgrad_remap_transposed_accumulate(T):
    # A rows remapped (drop one row per group of 5: the encoder's cls rows), output transposed, accumulate
    G, K0 = 4, 60
    a_full, b = _rnd(K0 // G * (G + 1), 64, seed=3), _rnd(K0, 48, seed=4)
    rows = torch.tensor([(k // G) * (G + 1) + 1 + k % G for k in range(K0)])
    ref = (a_full[rows].double().t() @ b.double()).float().t()
    out = torch.ones(48, 64, device="cuda")
    T.wgrad(a_full.cuda(), b.cuda(), 64, 48, K0, out, torch.float32, a_remap=(G, G + 1, 1), layout="dense_t",
            accumulate=True)
    torch.cuda.synchronize()
    check("_rel:out_1", _rel(out - 1, ref), 1e-5)


@pytest.mark.parametrize("M,N", [(768, 200), (72, 1000)])
def test_wgrad_remap_bf16(T, M, N):
    # the bf16 kernel's in-range address path on grouped rows (the encoder's 144 patch rows of every 145, cls
    # row first) on both operands; tile / split / column tails (M, N not multiples of the tiles)
    G, imgs = 144, 20
    K = G * imgs
    a_full, b_full = _rnd(imgs * (G + 1), M, seed=5), _rnd(imgs * (G + 1), N, seed=6)
    rows = torch.tensor([(k // G) * (G + 1) + 1 + k % G for k in range(K)])
    dt = torch.bfloat16
    ref = (a_full[rows].to(dt).double().t() @ b_full[rows].to(dt).double()).float()
    out = torch.empty(M, N, device="cuda")
    T.wgrad(a_full.cuda().to(dt), b_full.cuda().to(dt), M, N, K, out, dt, a_remap=(G, G + 1, 1),
            b_remap=(G, G + 1, 1))
    torch.cuda.synchronize()
    check("_rel:out", _rel(out, ref), 2e-3)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_wgrad_conv(T, stride, dt):
    n, H, cin, cout = 3, 12, 48, 40
    x = _rnd(n, cin, H, H, seed=5)
    Ho = (H + 2 - 3) // stride + 1
    dy = _rnd(n, cout, Ho, Ho, seed=6)
    xq, dyq = x.to(dt).float(), dy.to(dt).float()
    ref = torch.nn.grad.conv2d_weight(xq.double(), (cout, cin, 3, 3), dyq.double(), stride=stride, padding=1).float()
    x_nhwc = xq.permute(0, 2, 3, 1).contiguous().reshape(-1, cin).cuda().to(dt)
    dy_nhwc = dyq.permute(0, 2, 3, 1).contiguous().reshape(-1, cout).cuda().to(dt)
    out = torch.empty(cout, cin, 3, 3, device="cuda")
    T.wgrad(dy_nhwc, x_nhwc, cout, 9 * cin, n * Ho * Ho, out, dt, conv=dict(c1=cin, H=H, W=H, stride=stride, cin=cin),
            layout="conv")
    torch.cuda.synchronize()
    check("_rel:out", _rel(out, ref), (1e-5 if dt == torch.float32 else 2e-3))


@pytest.mark.parametrize("two_src", [False, True])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_wgrad_conv_batched(T, two_src, dt):
    """tmae_wgrad_args.nb: the weight (and bias) gradients of several same-shape 3x3 convs in ONE launch, each
    problem's dy / input / second input / output / bias at constant element strides (a shared input at stride 0,
    as the slices' first layers read LMS), every problem against its own f64 reference"""
    P, n, H, cin, cout = 4, 2, 12, 48, 40
    c2 = 16 if two_src else 0
    xs = [_rnd(n, cin - c2, H, H, seed=40 + j) for j in range(P)]
    xs[1] = xs[0] if two_src else xs[1]
    x2s = [_rnd(n, c2, H, H, seed=50 + j) for j in range(P)] if two_src else None
    dys = [_rnd(n, cout, H, H, seed=60 + j) for j in range(P)]
    q = lambda t: t.to(dt).float()  # noqa: E731
    nhwc = lambda t: q(t).permute(0, 2, 3, 1).contiguous().reshape(-1, t.shape[1])  # noqa: E731
    if two_src:  # the first input shared by every problem (stride 0), the second one per problem
        x1 = nhwc(xs[0]).cuda().to(dt)
        x2 = torch.stack([nhwc(t) for t in x2s]).cuda().to(dt)
        refs_x = [torch.cat([q(xs[0]), q(x2s[j])], 1) for j in range(P)]
    else:
        x1 = torch.stack([nhwc(t) for t in xs]).cuda().to(dt)
        refs_x = [q(xs[j]) for j in range(P)]
    dy = torch.stack([nhwc(t) for t in dys]).cuda().to(dt)
    out = torch.empty(P, cout, cin, 3, 3, device="cuda")
    bias = torch.empty(P, cout, device="cuda")
    npix = n * H * H
    conv = dict(c1=cin - c2, H=H, W=H, cin=cin, x2=x2[0] if two_src else None, ld2=c2)
    T.wgrad(dy[0], x1 if two_src else x1[0], cout, 9 * cin, npix, out[0], dt, conv=conv, layout="conv", bias=bias[0],
            ldb=cin - c2, batch=(P, npix * cout, 0 if two_src else npix * cin, npix * c2, cout * cin * 9, cout))
    torch.cuda.synchronize()
    for j in range(P):
        ref = torch.nn.grad.conv2d_weight(refs_x[j].double(), (cout, cin, 3, 3), q(dys[j]).double(), padding=1).float()
        check("_rel:batched_w", _rel(out[j], ref), (1e-5 if dt == torch.float32 else 2e-3))
        rb = q(dys[j]).double().sum((0, 2, 3)).float()
        check("_rel:batched_b", _rel(bias[j], rb), (1e-5 if dt == torch.float32 else 1e-4))


# bias gradient formed inside the weight-gradient GEMM (bf16: MFMAs against an all-ones fragment, one owner
# wave per fragment, folded in split order by tn_reduce; f32: column sums after the GEMM).  Shapes: one and
# many N tiles, M past the last whole M tile, more than 16 K splits (the 16 / 4-split fold), the 8-wave
# 256 x 256 tile, grouped rows, accumulation into an existing bias.
@pytest.mark.parametrize("K,M,N,remap", [(300, 72, 64, False), (9280, 72, 200, False), (1000, 200, 1000, False),
                                         (9280, 768, 3072, False), (2880, 768, 200, True), (16448, 520, 136, False)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("acc", [False, True])
def test_wgrad_bias(T, K, M, N, remap, dt, acc):
    if dt == torch.float32 and K * M * N > 3e9:
        pytest.skip("f32 parity path checked on the smaller shapes")
    if remap:
        G = 144
        imgs = K // G
        a_full, b_full = _rnd(imgs * (G + 1), M, seed=31), _rnd(imgs * (G + 1), N, seed=32)
        rows = torch.tensor([(k // G) * (G + 1) + 1 + k % G for k in range(K)])
        a, b = a_full[rows], b_full[rows]
        kw = dict(a_remap=(G, G + 1, 1), b_remap=(G, G + 1, 1))
        a_in, b_in = a_full, b_full
    else:
        a, b = _rnd(K, M, seed=33), _rnd(K, N, seed=34)
        kw = {}
        a_in, b_in = a, b
    ref_w = (a.to(dt).double().t() @ b.to(dt).double()).float()
    ref_b = a.to(dt).double().sum(0).float()
    out = torch.full((M, N), 0.25 if acc else 0.0, device="cuda")
    bias = torch.full((M,), 0.5 if acc else float("nan"), device="cuda")
    T.wgrad(a_in.cuda().to(dt), b_in.cuda().to(dt), M, N, K, out, dt, accumulate=acc, bias=bias, bias_accumulate=acc,
            **kw)
    torch.cuda.synchronize()
    off = 0.25 if acc else 0.0
    boff = 0.5 if acc else 0.0
    tol = 1e-5 if dt == torch.float32 else 2e-3
    check("_rel:w", _rel(out - off, ref_w), tol)
    # per element (a wrong fragment owner or split fold shows up as whole wrong columns, not as aggregate noise)
    db = (bias.cpu().double() - boff - ref_b.double()).abs()
    scale = a.to(dt).double().abs().sum(0)
    worst = float((db / scale.clamp_min(1e-30)).max())
    check("_rel:bias_per_elem", worst, 1e-6 if dt == torch.float32 else 1e-5)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_wgrad_conv_bias(T, dt):
    # the conv layout with the bias column sums of dy (the conv's bias gradient)
    n, H, cin, cout = 4, 12, 48, 40
    x, dy = _rnd(n, cin, H, H, seed=35), _rnd(n, cout, H, H, seed=36)
    xq, dyq = x.to(dt).float(), dy.to(dt).float()
    ref = torch.nn.grad.conv2d_weight(xq.double(), (cout, cin, 3, 3), dyq.double(), padding=1).float()
    ref_b = dyq.double().sum((0, 2, 3))
    x_nhwc = xq.permute(0, 2, 3, 1).contiguous().reshape(-1, cin).cuda().to(dt)
    dy_nhwc = dyq.permute(0, 2, 3, 1).contiguous().reshape(-1, cout).cuda().to(dt)
    out = torch.empty(cout, cin, 3, 3, device="cuda")
    bias = torch.empty(cout, device="cuda")
    T.wgrad(dy_nhwc, x_nhwc, cout, 9 * cin, n * H * H, out, dt, conv=dict(c1=cin, H=H, W=H, cin=cin), layout="conv",
            bias=bias)
    torch.cuda.synchronize()
    check("_rel:w", _rel(out, ref), 1e-5 if dt == torch.float32 else 2e-3)
    db = (bias.cpu().double() - ref_b).abs() / dyq.double().abs().sum((0, 2, 3))
    check("_rel:bias_per_elem", float(db.max()), 1e-6 if dt == torch.float32 else 1e-5)


def test_wgrad_conv_two_sources(T):
    # torch.cat([x1, x2], 1) without a copy, written into a channel slice of a wider weight
    n, H, c1, c2, cout = 2, 6, 16, 8, 24
    x1, x2, dy = _rnd(n, c1, H, H, seed=7), _rnd(n, c2, H, H, seed=8), _rnd(n, cout, H, H, seed=9)
    ref = torch.nn.grad.conv2d_weight(torch.cat([x1, x2], 1).double(), (cout, c1 + c2, 3, 3), dy.double(),
                                      padding=1).float()
    out = torch.zeros(cout, c1 + c2 + 8, 3, 3, device="cuda")
    nh = lambda t: t.permute(0, 2, 3, 1).contiguous().reshape(-1, t.shape[1]).cuda()  # noqa: E731
    T.wgrad(nh(dy), nh(x1), cout, 9 * (c1 + c2), n * H * H, out, torch.float32,
            conv=dict(x2=nh(x2), c1=c1, ld2=c2, H=H, W=H, cin=c1 + c2), layout="conv", cin_total=c1 + c2 + 8,
            ci_off=8)
    torch.cuda.synchronize()
    assert _rel(out[:, 8:], ref) < 1e-5 and out[:, :8].abs().max().item() == 0


# ------------------------------------------------------------------------------ data gradients
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_dgrad_linear_gelu(T, dt):
    M, N, K = 290, 256, 136
    dy, w, pre = _rnd(M, N, seed=10), _rnd(N, K, seed=11) / 16, _rnd(M, K, seed=12)
    dyq, wq, preq = dy.to(dt).float(), w.to(dt).float(), pre.to(dt).float()
    x = preq.clone().requires_grad_(True)
    (F.gelu(x) * (dyq @ wq)).sum().backward()
    ref = x.grad
    wt = wq.t().contiguous().cuda().to(dt)
    out = torch.empty(M, K, device="cuda", dtype=torch.float32)
    T.dgrad_linear(dyq.cuda().to(dt), wt, M, N, K, dt, out=out, pre=preq.cuda().to(dt))
    acc = torch.ones(M, K, device="cuda")
    T.dgrad_linear(dyq.cuda().to(dt), wt, M, N, K, dt, acc32=acc)
    torch.cuda.synchronize()
    tol = 1e-4 if dt == torch.float32 else 1e-2
    check("_rel:out", _rel(out, ref), tol)
    check("_rel:acc_1", _rel(acc - 1, dyq @ wq), tol)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_conv_dgrad(T, stride, dt):
    n, H, cin, cout = 2, 12, 40, 48
    Ho = (H + 2 - 3) // stride + 1
    w, dy, pre = _rnd(cout, cin, 3, 3, seed=13) / 8, _rnd(n, cout, Ho, Ho, seed=14), _rnd(n, cin, H, H, seed=15)
    wq, dyq, preq = w.to(dt).float(), dy.to(dt).float(), pre.to(dt).float()
    dx = torch.nn.grad.conv2d_input((n, cin, H, H), wq.double(), dyq.double(), stride=stride, padding=1).float()
    x = preq.clone().requires_grad_(True)
    (F.gelu(x) * dx).sum().backward()
    nh = lambda t: t.permute(0, 2, 3, 1).contiguous().reshape(-1, t.shape[1])  # noqa: E731
    wd = wq.permute(1, 2, 3, 0).contiguous().reshape(cin, -1).cuda().to(dt)
    out = torch.empty(n * H * H, cin, device="cuda")
    T.conv_dgrad(nh(dyq).cuda().to(dt), wd, n, H, H, stride, cout, cin, dt, out=out, pre=nh(preq).cuda().to(dt))
    # routed f32 accumulation of the same data gradient: channels [0,16) / [16,24) / [24,40)
    r0, r1, r2 = (torch.ones(n * H * H, c, device="cuda") for c in (16, 8, 16))
    T.conv_dgrad(nh(dyq).cuda().to(dt), wd, n, H, H, stride, cout, cin, dt, routes=[(r0, 16, 16), (r1, 8, 8), (r2, 16, 16)])
    torch.cuda.synchronize()
    tol = 1e-4 if dt == torch.float32 else 1e-2
    check("_rel:out", _rel(out, nh(x.grad)), tol)
    check("_rel:torch_cat_r0_r1_r2_1_1", _rel(torch.cat([r0, r1, r2], 1) - 1, nh(dx)), tol)


def test_layernorm_bwd_remap(T):
    B, Tn, D = 3, 7, 128
    x = _rnd(B * Tn, D, seed=16)
    gamma, beta = 1 + 0.1 * _rnd(D, seed=17), 0.1 * _rnd(D, seed=18)
    rows = torch.tensor([b * Tn + 1 + k for b in range(B) for k in range(Tn - 1)])  # drop cls rows
    dy = _rnd(len(rows), D, seed=19)
    xr, g_, b_ = x.clone().requires_grad_(True), gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    (F.layer_norm(xr[rows], (D,), g_, b_, 1e-6) * dy).sum().backward()
    dres = _rnd(B * Tn, D, seed=20)
    dx = torch.zeros(B * Tn, D, device="cuda")
    dxop = torch.zeros(B * Tn, D, device="cuda", dtype=torch.bfloat16)
    dg, db, drs = torch.empty(D, device="cuda"), torch.empty(D, device="cuda"), torch.empty(D, device="cuda")
    T.layernorm_bwd(x.cuda(), gamma.cuda(), dy.cuda(), dx, len(rows), D, 1e-6, dg, db, dres=dres.cuda(), dxop=dxop,
                    row_group=Tn - 1, group_stride=Tn, row_offset=1, dres_colsum=drs)
    torch.cuda.synchronize()
    check("_rel:drs", _rel(drs, dres[rows].sum(0)), 1e-5)  # bias gradient of the residual's Linear, folded in
    ref = xr.grad.clone()
    ref[rows] += dres[rows]
    check("_rel:dx", _rel(dx, ref), 1e-5)
    check("_rel:dxop_float", _rel(dxop.float(), ref), 6e-3)
    assert _rel(dg, g_.grad) < 1e-5 and _rel(db, b_.grad) < 1e-5


# ------------------------------------------------------------------------------ attention
@pytest.mark.parametrize("T_,H,dh", [(145, 12, 64), (257, 16, 32), (20, 2, 64), (65, 4, 80), (161, 2, 80), (32, 2, 32),
                                     (33, 3, 32), (288, 4, 32), (160, 2, 64), (1, 2, 32)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_mha_bwd(T, T_, H, dh, dt):
    from textmae_amd import ops

    B = 2
    D = H * dh
    qkv = _rnd(B * T_, 3 * D, seed=21).to(dt).float()
    do = _rnd(B * T_, D, seed=22).to(dt).float()
    scale = dh ** -0.5
    q_ = qkv.clone().requires_grad_(True)
    t = q_.reshape(B, T_, 3, H, dh).permute(2, 0, 3, 1, 4)
    att = ((t[0] @ t[1].transpose(-2, -1)) * scale).softmax(-1)
    o = (att @ t[2]).transpose(1, 2).reshape(B * T_, D)
    (o * do).sum().backward()
    qg = qkv.cuda().to(dt)
    out = torch.empty(B * T_, D, device="cuda", dtype=dt)
    lse = torch.empty(B * H * T_, device="cuda")
    T.mha_lse(qg, B, T_, H, dh, scale, dt, out, lse)
    dq = torch.empty(B * T_, 3 * D, device="cuda", dtype=dt)
    T.mha_bwd(qg, out, do.cuda().to(dt), lse, dq, B, T_, H, dh, scale, dt)
    dq2 = torch.empty_like(dq)
    T.mha_bwd(qg, out, do.cuda().to(dt), lse, dq2, B, T_, H, dh, scale, dt)
    o_plain = ops.mha(qg, B, T_, H, dh, scale, dt)
    torch.cuda.synchronize()
    assert torch.equal(dq, dq2)  # fixed summation order: bitwise reproducible
    assert torch.equal(out, o_plain)  # the lse variant computes the same output
    if dt == torch.float32:
        check("_rel:out", _rel(out, o), 1e-5)
        check("_rel:dq", _rel(dq, q_.grad), 1e-4)
    else:
        check("_rel2:dq_float", _rel2(dq.float(), q_.grad), 5e-3)


# ------------------------------------------------------------------------------ distortion
@pytest.mark.parametrize("hw", [(40, 37), (100, 150), (256, 256), (100, 152, "offset")])
def test_distortion_fwd_bwd_vs_oracle(hw):
    """one tile, several 32 x 64 tiles with ragged edges, the bench's 256^2 (tiled kernels, distortion.hip); and
    inputs that are contiguous views 4 B past a 16-B boundary (a sliced batch), which must take the per-element
    path of the backward's 16-B accesses"""
    from oracle.thirdparty import ssim as ssim_ref
    from textmae_amd.distortion import ssim_l1_loss

    H, W = hw[:2]
    offset = len(hw) > 2
    x = torch.rand(2, 3, H, W, generator=torch.Generator().manual_seed(30))
    y = (x + 0.1 * _rnd(2, 3, H, W, seed=31)).clamp(0, 1)
    xr = x.double().requires_grad_(True)
    s_ref = 1 - ssim_ref(xr, y.double(), data_range=1)
    l_ref = F.l1_loss(xr, y.double())
    (0.7 * s_ref + 1.3 * l_ref).backward()
    if offset:  # 1-float offset views: base pointers 4 B past a 16-B boundary
        xb = torch.empty(x.numel() + 1, device="cuda")
        yb = torch.empty(y.numel() + 1, device="cuda")
        xg, yd = xb[1:].view_as(x), yb[1:].view_as(y)
        xg.copy_(x)
        yd.copy_(y)
        assert xg.data_ptr() % 16 and yd.data_ptr() % 16
        xg.requires_grad_(True)
    else:
        xg, yd = x.cuda().requires_grad_(True), y.cuda()
    s, l = ssim_l1_loss(xg, yd)
    (0.7 * s + 1.3 * l).backward()
    torch.cuda.synchronize()
    assert abs(s.item() - s_ref.item()) < 1e-5 and abs(l.item() - l_ref.item()) < 1e-6
    check("_rel:xg_grad", _rel(xg.grad, xr.grad), 1e-4)


# ------------------------------------------------------------------------------ optimizer
def test_adam_matches_torch(T):
    n = 1000
    p0, g = _rnd(n, seed=23), _rnd(n, seed=24)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3, weight_decay=0.01)
    p, m, v = p0.cuda(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
    clip = torch.tensor([0.5, 0.5], device="cuda")
    for step in range(1, 4):
        ref.grad = g * 0.5
        opt.step()
        T.adam(p, g.cuda(), m, v, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, clip=clip[1:])
    norm = torch.empty(2, device="cuda")
    T.grad_norm(g.cuda(), 1.0, norm)
    torch.cuda.synchronize()
    check("_rel:p", _rel(p, ref.detach()), 1e-6)
    assert abs(norm[0].item() - g.norm().item()) < 1e-4 * g.norm().item()
    assert abs(norm[1].item() - min(1.0, 1.0 / (g.norm().item() + 1e-6))) < 1e-6


@pytest.mark.parametrize("n,off", [(3_000_013, 0), (1_048_576 + 5, 1)])
def test_grad_norm_and_scale_vector_paths(T, n, off):
    # the 16-B paths of the norm and the in-place scale, a ragged tail, and an unaligned buffer (off = 1 float)
    g0 = _rnd(n + off, seed=25)
    buf = g0.cuda()
    g = buf[off:]
    norm = torch.empty(2, device="cuda")
    T.grad_norm(g, 0.5, norm)
    T.scale_(g, norm[1:])
    torch.cuda.synchronize()
    ref = g0[off:].double().norm().item()
    assert abs(norm[0].item() - ref) < 1e-5 * ref
    assert torch.equal(buf[off:].cpu(), g0[off:] * norm[1].item())
    assert torch.equal(buf[:off].cpu(), g0[:off])


# ------------------------------------------------------------------------------ whole model
SMALL = dict(img_size=64, patch_size=16, encoder_embed_dim=64, encoder_depth=2, encoder_num_heads=2,
             decoder_embed_dim=64, decoder_depth=2, decoder_num_heads=2, latent_depth=192, hyperprior_depth=96,
             num_slices=12, num_keep_patches=16)


def _model_and_oracle(cfgd, seed, B, dt):
    import textmae_amd
    from oracle.mcm_oracle import MCMConfig, make_state_dict

    cfg = MCMConfig(**cfgd)
    sd = make_state_dict(cfg, seed)
    m = textmae_amd.MCM(**cfg.kwargs())
    full = m.state_dict()
    full.update(sd)
    m.load_state_dict(full)
    m = m.cuda().train()
    m.compute_dtype = dt
    m.distortion = "none"
    rng = np.random.default_rng(seed + 1)
    L = (cfg.img_size // cfg.patch_size) ** 2
    g = int(cfg.num_keep_patches ** 0.5)
    hz = g // 4
    imgs = torch.from_numpy(rng.random((B, 3, cfg.img_size, cfg.img_size), dtype=np.float32))
    scores = torch.from_numpy(rng.random((B, L), dtype=np.float32))
    zn = torch.from_numpy(rng.uniform(-0.5, 0.5, (B, cfg.hyperprior_depth, hz, hz)).astype(np.float32))
    yn = torch.from_numpy(rng.uniform(-0.5, 0.5, (B, cfg.latent_depth, g, g)).astype(np.float32))
    R = torch.from_numpy(rng.standard_normal((B, 3, cfg.img_size, cfg.img_size)).astype(np.float32)) * 1e-2
    return m, cfg, sd, imgs, scores, zn, yn, R


def _hip_grads(m, imgs, scores, zn, yn, R):
    from textmae_amd.rd_loss import RateDistortionLoss

    m.zero_grad(set_to_none=True)
    out = m(imgs.cuda(), scores.cuda(), noise=(zn.cuda(), yn.cuda()))
    crit = RateDistortionLoss(lmbda=1e-2)
    loss = crit(out, imgs.cuda())["bpp_loss"] + (out["x_hat"] * R.cuda()).sum()
    loss.backward()
    aux = m.aux_loss()
    aux.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters() if p.requires_grad}, out, loss, aux


def _oracle_grads(cfg, sd, imgs, scores, zn, yn, R):
    from oracle.train_oracle import aux_loss, mcm_forward_train, rate_bpp

    leaf = {k: (v.clone().double().requires_grad_(True) if torch.is_floating_point(v) and not k.endswith("pos_embed")
                and k != "entropy_bottleneck.target" else (v.double() if torch.is_floating_point(v) else v))
            for k, v in sd.items()}
    x_hat, ylik, zlik = mcm_forward_train(leaf, cfg, imgs.double(), scores, zn.double(), yn.double())
    n, _, H, W = imgs.shape
    loss = rate_bpp(ylik, zlik, n * H * W) + (x_hat * R.double()).sum()
    loss.backward()
    aux = aux_loss(leaf, "entropy_bottleneck.")
    aux.backward()
    return {k: v.grad for k, v in leaf.items() if isinstance(v, torch.Tensor) and v.requires_grad}, x_hat, loss, aux


def test_mcm_train_grads_f32_vs_oracle():
    m, cfg, sd, imgs, scores, zn, yn, R = _model_and_oracle(SMALL, 3, 2, torch.float32)
    hip, out, loss, aux = _hip_grads(m, imgs, scores, zn, yn, R)
    ref, x_ref, loss_ref, aux_ref = _oracle_grads(cfg, sd, imgs, scores, zn, yn, R)
    check("_rel:out_x_hat", _rel(out["x_hat"], x_ref), 1e-4)
    assert abs(loss.item() - loss_ref.item()) < 1e-4 * max(1.0, abs(loss_ref.item()))
    assert abs(aux.item() - aux_ref.item()) < 1e-4 * abs(aux_ref.item())
    bad = []
    for name, g in hip.items():
        r = ref[name].float()
        if r.abs().max() == 0:
            if g.abs().max() > 1e-6:
                bad.append((name, "nonzero", g.abs().max().item()))
            continue
        e = _rel(g, r)
        if e > 2e-3:
            bad.append((name, e))
    assert not bad, bad[:20]


def test_mcm_train_bf16_close_to_f32():
    m, cfg, sd, imgs, scores, zn, yn, R = _model_and_oracle(SMALL, 4, 2, torch.float32)
    g32, *_ = _hip_grads(m, imgs, scores, zn, yn, R)
    m.compute_dtype = torch.bfloat16
    g16, *_ = _hip_grads(m, imgs, scores, zn, yn, R)
    flat32 = torch.cat([g32[k].reshape(-1) for k in g32])
    flat16 = torch.cat([g16[k].reshape(-1) for k in g32])
    assert torch.isfinite(flat16).all()
    check("_rel2:flat16", _rel2(flat16, flat32), 3e-3)


@pytest.mark.parametrize("geom", ["small", "vitb"])
def test_train_fused_stacks_vs_per_layer(geom):
    """the bf16 training forward's slice stacks on tmae_lic_stack (latent partial sums + chained / batched stacks
    keeping every layer's pre-activation and output) against the same model on the per-layer conv launches: outputs
    and every gradient within the bf16 rounding of the different summation order"""
    from textmae_amd.mcm_train import TrainExec

    cfgd = SMALL if geom == "small" else dict(img_size=256, num_keep_patches=144)
    B = 2 if geom == "small" else 4
    m, cfg, sd, imgs, scores, zn, yn, R = _model_and_oracle(cfgd, 9, B, torch.bfloat16)
    res = {}
    for fused in (True, False):
        TrainExec.USE_LIC_STACK = fused
        try:
            m._train_exec = None
            g, out, loss, aux = _hip_grads(m, imgs, scores, zn, yn, R)
            assert m._train_exec._fused_ok() == fused
        finally:
            TrainExec.USE_LIC_STACK = True
        res[fused] = (g, out["x_hat"].float().cpu(), out["likelihoods"]["y"].float().cpu())
    (ga, xa, ya), (gb, xb, yb) = res[True], res[False]
    check(f"_rel2:fused_train_x_hat_{geom}", _rel2(xa, xb), 2e-2)
    check(f"_rel2:fused_train_ylik_{geom}", _rel2(ya, yb), 2e-2)
    fa = torch.cat([ga[k].reshape(-1) for k in ga])
    fb = torch.cat([gb[k].reshape(-1) for k in ga])
    assert torch.isfinite(fa).all()
    check(f"_rel2:fused_train_grads_{geom}", _rel2(fa, fb), 3e-2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_side_stream_wgrads_bitwise(dt):
    """weight gradients on the side stream (mcm_train._wg, deferred one-per-group forks) == the same backward
    with every weight gradient on the compute stream, bit for bit; and the side stream really ran them"""
    m, cfg, sd, imgs, scores, zn, yn, R = _model_and_oracle(SMALL, 5, 3, dt)
    g_side, *_ = _hip_grads(m, imgs, scores, zn, yn, R)
    ex = m._train_exec
    assert ex.__dict__.get("_side") is not None and ex._side_calls > 0
    ex._side = None  # _side_begin keeps an instance attribute: None = every weight gradient on the compute stream
    g_one, *_ = _hip_grads(m, imgs, scores, zn, yn, R)
    assert ex._side_calls == 0
    bad = [k for k in g_side if not torch.equal(g_side[k], g_one[k])]
    assert not bad, bad[:10]


def _partial_loss_grads(m, imgs, scores, zn, yn, R, nsel):
    """HIP backward of a loss over the first `nsel` images only (rate of those images + sum(x_hat * R)), run
    at the batch of `imgs`: images never mix, so the gradient equals that of the same loss on a batch of
    `nsel` -- which lets the oracle check the bench batch's tile / split-K geometry on a small sample"""
    m.zero_grad(set_to_none=True)
    out = m(imgs.cuda(), scores.cuda(), noise=(zn.cuda(), yn.cuda()))
    n, _, H, W = imgs.shape
    ylik, zlik = out["likelihoods"]["y"], out["likelihoods"]["z"]
    loss = ((torch.log(ylik[:nsel]).sum() + torch.log(zlik[:nsel]).sum()) / (-math.log(2) * nsel * H * W)
            + (out["x_hat"] * R.cuda()).sum())
    loss.backward()
    aux = m.aux_loss()
    aux.backward()
    torch.cuda.synchronize()
    return {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters() if p.requires_grad}, out, loss, aux


def test_mcm_train_grads_vitb_batch64_f32_vs_oracle():
    """north-star geometry (ViT-B/16 256^2, K=144) at the bench's batch of 64, f32 parity path: the whole
    model's parameter gradients against the autograd oracle (f64) for a loss over images 0-1 (injected
    noise), i.e. the batch-64 tile / split-K choices and bias-sum folds composed over 12 + 8 blocks"""
    B, NS = 64, 2
    m, cfg, sd, imgs, scores, zn, yn, R = _model_and_oracle(dict(img_size=256, num_keep_patches=144), 7, B,
                                                            torch.float32)
    R[NS:] = 0
    hip, out, loss, aux = _partial_loss_grads(m, imgs, scores, zn, yn, R, NS)
    torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
    ref, x_ref, loss_ref, aux_ref = _oracle_grads(cfg, sd, imgs[:NS], scores[:NS], zn[:NS], yn[:NS], R[:NS])
    check("_rel:x_hat_vitb", _rel(out["x_hat"][:NS], x_ref), 1e-4)
    check("loss_rel_vitb", abs(loss.item() - loss_ref.item()) / max(1.0, abs(loss_ref.item())), 1e-4)
    worst, bad = 0.0, []
    for name, g in hip.items():
        r = ref[name].float()
        if r.abs().max() == 0:
            if g.abs().max() > 1e-6:
                bad.append((name, "nonzero", g.abs().max().item()))
            continue
        e = _rel(g, r)
        worst = max(worst, e)
        if e > 1e-5:
            bad.append((name, e))
    check("grad_maxrel_worst_tensor_vitb_b64_f32", worst, 1e-5, tensors=len(hip))  # measured 3.5e-6
    assert not bad, bad[:20]
    # the benched operand dtype at the same batch against these f32 gradients
    m.compute_dtype = torch.bfloat16
    g16, *_ = _partial_loss_grads(m, imgs, scores, zn, yn, R, NS)
    flat32 = torch.cat([hip[k].reshape(-1) for k in hip])
    flat16 = torch.cat([g16[k].reshape(-1) for k in hip])
    assert torch.isfinite(flat16).all()
    check("grad_relL2_bf16_vs_f32_vitb_b64", _rel2(flat16, flat32), 1e-2)  # measured 5.1e-3


def test_mcm_train_vitb_step_runs():
    """north-star geometry (ViT-B/16 256^2, K=144) at a small batch: fwd + bwd + 2 Adam steps, bf16"""
    import textmae_amd
    from textmae_amd.optim import FusedAdam
    from textmae_amd.rd_loss import RateDistortionLoss

    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
    m.compute_dtype = torch.bfloat16
    opt = FusedAdam([p for n, p in m.named_parameters() if not n.endswith(".quantiles")], lr=1e-4)
    imgs = torch.rand(2, 3, 256, 256, device="cuda")
    scores = torch.rand(2, 256, device="cuda")
    crit = RateDistortionLoss(lmbda=1e-2)
    losses = []
    for _ in range(2):
        out = m(imgs, scores)
        loss = crit(out, imgs)["loss"]
        opt.zero_grad()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
        opt.step()
        losses.append(loss.item())
    assert all(math.isfinite(v) for v in losses)
    assert all(torch.isfinite(p).all() for p in m.parameters())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_relayout_multi_dense_and_strided(T, dt):
    """tmae_relayout_multi (the weight cache's one launch per optimizer step): plain casts (vector path,
    ragged tails, an unaligned destination) and strided permutes in one table, exact against torch"""
    from textmae_amd import _lib, ops

    dev = "cuda"
    srcs = [_rnd(5000, seed=1), _rnd(64, 3, 3, 40, seed=2), _rnd(32768 * 2 + 8200, seed=3), _rnd(96, 130, seed=4),
            _rnd(32768 * 2 + 7, seed=5)]
    srcs = [s.to(dev) for s in srcs]
    big = torch.empty(32768 * 2 + 8, dtype=dt, device=dev)
    jobs = [  # (source, destination, dims, element strides)
        (srcs[0], torch.empty(5000, dtype=dt, device=dev), (5000,), (1,)),
        (srcs[1], torch.empty(64, 40, 3, 3, dtype=dt, device=dev), (64, 40, 3, 3), (360, 1, 120, 40)),
        # 3 chunks, the last one ragged inside its second 8192-element round
        (srcs[2], torch.empty(32768 * 2 + 8200, dtype=dt, device=dev), (32768 * 2 + 8200,), (1,)),
        (srcs[3], torch.empty(130, 96, dtype=dt, device=dev), (130, 96), (1, 130)),
        (srcs[4], big[1:], (32768 * 2 + 7,), (1,)),   # destination 2 or 4 B past a 16-B boundary
    ]
    rows, chunk = [], 0
    for s, d, dims, st in jobs:
        dd = list(dims) + [1] * (4 - len(dims))
        ss = list(st) + [0] * (4 - len(st))
        total = dd[0] * dd[1] * dd[2] * dd[3]
        rows.append([s.data_ptr(), d.data_ptr(), ops.dtype_code(dt), dd[1], dd[2], dd[3], *ss, total, chunk])
        chunk += (total + 32767) // 32768
    owner = [t for t, r in enumerate(rows) for _ in range((rows[t + 1][11] if t + 1 < len(rows) else chunk) - r[11])]
    tab = torch.tensor([v for r in rows for v in r] + owner, dtype=torch.int64).to(dev)
    _lib.call("tmae_relayout_multi", tab.data_ptr(), len(rows), chunk, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for s, d, dims, st in jobs:
        ref = torch.as_strided(s, dims, st).to(dt)
        assert torch.equal(d.reshape(dims), ref)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_weight_cache_refresh_modes(dt):
    """mcm_train._Weights: the lazy first build and the one-launch refresh (tmae_relayout_multi modes: plain
    cast, 64 x 64 LDS transposes for W^T and the conv data-gradient layout, per-row [Cin][9] -> [9][Cin] for conv
    weights) equal torch's layouts exactly, including ragged transpose edges"""
    from textmae_amd.mcm_train import _Weights
    from textmae_amd.optim import bump_versions

    g = torch.Generator().manual_seed(7)
    lin = torch.nn.Parameter(torch.randn(200, 136, generator=g).cuda())
    conv = torch.nn.Parameter(torch.randn(72, 40, 3, 3, generator=g).cuda())
    conv2 = torch.nn.Parameter(torch.randn(32, 608, 3, 3, generator=g).cuda())
    W = _Weights(dt)

    def check_all():
        torch.cuda.synchronize()
        assert torch.equal(W.nt(lin), lin.detach().to(dt))
        assert torch.equal(W.t(lin), lin.detach().t().contiguous().to(dt))
        for c in (conv, conv2):
            co, ci = c.shape[:2]
            assert torch.equal(W.conv(c), c.detach().permute(0, 2, 3, 1).reshape(co, 9 * ci).to(dt))
            assert torch.equal(W.conv_dg(c), c.detach().permute(1, 2, 3, 0).reshape(ci, 9 * co).to(dt))

    # packed kinds of the fused training stacks: conv_dg problems back to back, the fragment order of
    # tmae_lic_stack over an input-channel range (relayout mode 3), the latent-channel slice in conv layout
    convb = torch.nn.Parameter(torch.randn(72, 40, 3, 3, generator=g).cuda())
    from textmae_amd import ops

    def check_packs():
        torch.cuda.synchronize()
        dg = W.packed([conv, convb], "conv_dg")
        for j, c in enumerate((conv, convb)):
            assert torch.equal(dg[j], c.detach().permute(1, 2, 3, 0).reshape(40, 9 * 72).to(dt))
        # (2, 16): source rows not 16-B aligned (the scalar path of mode 3)
        for lo, n in ((8, 24), (0, 40), (16, 0), (2, 16)):
            pk = W.packed([conv, convb], ("lic", lo, n))
            for j, c in enumerate((conv, convb)):
                assert torch.equal(pk[j], ops.pack_lic_stack_weight(c.detach()[:, lo:lo + n], dt)), (lo, n)
        # the transposed, tap-flipped pack (mode 4): 72 -> 3 ragged k-steps, 40 -> 3 ragged fragments
        pt = W.packed([conv, convb], "licT")
        for j, c in enumerate((conv, convb)):
            assert torch.equal(pt[j], ops.pack_lic_stack_weight_t(c.detach(), dt))
        lat = W.packed([conv, convb], ("conv_lat", 24))
        for j, c in enumerate((conv, convb)):
            assert torch.equal(lat[j], c.detach()[:, :24].permute(0, 2, 3, 1).reshape(72, 9 * 24).to(dt))

    check_all()  # lazy first builds
    check_packs()
    with torch.no_grad():
        for p in (lin, conv, conv2, convb):
            p.mul_(-1.5).add_(0.25)
    bump_versions([lin, conv, conv2, convb])
    W.refresh()  # one multi-tensor launch
    torch.cuda.synchronize()
    # the cached copies are returned as-is now (signatures current): they must hold the new values
    check_all()
    check_packs()
