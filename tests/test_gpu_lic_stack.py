"""tmae_lic_stack (csrc/lic_stack.hip): a whole slice-transform stack (cc_transform_mean / _scale /
lrp_transform, MCM.py:165-293 applied at MCM.py:761-784) per workgroup.

* the kernel against a plain PyTorch fp32 restatement of the same stack (conv2d + GELU chain over
  bf16-rounded operands, activations rounded to bf16 between layers as the kernel stores them in LDS):
  two input sources (torch.cat without a copy), the layer-0 addend, batched problems with strides, the
  f32 (mu / sigma) and the lrp (y_hat_pre + 0.5 tanh) outputs, the 12x12 and 8x8 grids, an empty
  layer-0 input (slice 0's mean / scale stacks);
* the MCM eval forward with the fused stacks against the layer-by-layer launches (_Executor.USE_LIC_STACK) on
  the same weights, bf16, at the benched geometry.
Tolerance: bf16 operands, f32 accumulation -> max|a-b| / max|b| <= 6e-3 per output (2x the measured 3.0e-3).
"""
import pytest
import torch
import torch.nn.functional as F
from parity_log import check, record

pytestmark = pytest.mark.gpu
DEV = "cuda"
MID = [224, 176, 128, 80, 32]
STACK_MAXREL = 6e-3  # bf16 operands; about 2x the largest measured error, 3.0e-3 (profiles/r03/parity_metrics.jsonl)


def _bf(t):
    return t.to(torch.bfloat16).float()


def _ref_stack(x, ws, bs, G, addend=None, lrp_src=None):
    """x [P][n*G*G][cin0] f32 (bf16 values); ws[l] [P][Cout][Cin][3][3]; returns [P][n*G*G][Cout_last]"""
    P, rows, cin0 = x.shape
    n = rows // (G * G)
    outs = []
    for p in range(P):
        h = x[p].view(n, G, G, cin0).permute(0, 3, 1, 2)
        for l, (w, b) in enumerate(zip(ws, bs)):
            h = F.conv2d(h, w[p], b[p], padding=1) if w[p].shape[1] else b[p].view(1, -1, 1, 1).expand(n, -1, G, G)
            if l == 0 and addend is not None:
                h = h + addend[p].view(n, G, G, -1).permute(0, 3, 1, 2)
            if l + 1 < len(ws):
                h = _bf(F.gelu(h))
        h = h.permute(0, 2, 3, 1).reshape(rows, -1)
        if lrp_src is not None:
            h = lrp_src[p] + 0.5 * torch.tanh(h)
        outs.append(h)
    return torch.stack(outs)


def _maxrel(a, b):
    return float((a.double() - b.double()).abs().max() / b.double().abs().max())


@pytest.mark.parametrize("G,c1,c2,nb,mode", [
    (12, 64, 32, (2, 3), "f32"),
    (12, 160, 0, (2, 1), "f32"),
    (12, 0, 0, (2, 1), "f32"),
    (12, 192, 32, (1, 2), "lrp"),
    (8, 96, 0, (1, 1), "lrp"),
])
def test_lic_stack_vs_torch(tmae, G, c1, c2, nb, mode):
    from textmae_amd import ops

    torch.manual_seed(G * 1000 + c1 + c2)
    n, P = 5, nb[0] * nb[1]
    rows = n * G * G
    cin0 = c1 + c2
    ld1, ld2 = c1 + 16, c2 + 8
    x1 = torch.randn(rows, ld1).to(torch.bfloat16).to(DEV)
    x2 = torch.randn(P, rows, ld2).to(torch.bfloat16).to(DEV)  # one slab per problem (s2 for b2, s1 for b1)
    chans = [cin0] + MID
    ws = [_bf(torch.randn(P, chans[l + 1], chans[l], 3, 3) / (3.0 * max(chans[l], 1) ** 0.5)) for l in range(5)]
    bs = [torch.randn(P, c) * 0.1 for c in MID]
    add = torch.randn(P, rows, 240) * 0.5
    packed = [torch.stack([ops.pack_lic_stack_weight(w[p]) for p in range(P)]).to(DEV) for w in ws]
    bias = [b.contiguous().to(DEV) for b in bs]
    addd = add.to(DEV)
    st = {"x2": (nb[1] * rows * ld2, rows * ld2), "a": (nb[1] * rows * 240, rows * 240)}
    for l in range(5):
        sz = packed[l][0].numel()
        st[f"w{l}"] = (nb[1] * sz, sz)
        st[f"b{l}"] = (nb[1] * MID[l], MID[l])
    x_in = torch.cat([x1[:, :c1].float().cpu().expand(P, -1, -1), x2[:, :, :c2].float().cpu()], dim=2)
    if mode == "f32":
        y = torch.zeros(P, rows, 40, device=DEV)
        st["y"] = (nb[1] * rows * 40, rows * 40)
        ops.lic_stack(n, G, x1, c1, ld1, packed, bias, MID, y, 40, True, x2=x2 if c2 else None, c2=c2, ld2=ld2,
                      addend=addd, ld_add=240, nb=nb, strides=st)
        ref = _ref_stack(x_in, ws, bs, G, addend=add[:, :, :224])
        got = y[:, :, :32].cpu()
    else:
        src = torch.randn(P, rows, 48)
        y = torch.zeros(P, rows, 48, dtype=torch.bfloat16, device=DEV)
        y2 = torch.zeros_like(y)
        st.update({"y": (nb[1] * rows * 48, rows * 48), "src": (nb[1] * rows * 48, rows * 48),
                   "y2": (nb[1] * rows * 48, rows * 48)})
        ops.lic_stack(n, G, x1, c1, ld1, packed, bias, MID, y, 48, False, x2=x2 if c2 else None, c2=c2, ld2=ld2,
                      addend=addd, ld_add=240, lrp_src=src.to(DEV), ld_src=48, y2=y2, ldy2=48, nb=nb, strides=st)
        ref = _ref_stack(x_in, ws, bs, G, addend=add[:, :, :224], lrp_src=src[:, :, :32])
        got = y[:, :, :32].float().cpu()
        assert torch.equal(y, y2)
        assert float(y[:, :, 32:].float().abs().max()) == 0.0  # nothing outside the 32 output channels
    torch.cuda.synchronize()
    err = _maxrel(got, ref)
    print(f"G={G} cin={c1}+{c2} nb={nb} {mode}: max rel err {err:.2e}")
    check(f"lic_stack_maxrel_{mode}", err, STACK_MAXREL)


LATENT_MAXREL = 1e-5  # f32 sums of bf16 products in another order than conv2d: ~10x the measured 1.1e-6


@pytest.mark.parametrize("G,cin,nfr,nblk,nb,f_lo,f_hi", [
    (12, 384, 14, 36, 3, 14, 28),    # the bench geometry: slice 1's mean / lrp / scale blocks
    (12, 384, 14, 36, 3, 84, 168),   # slices 6..11 (6 tiles of 16 fragments, the last one partial)
    (12, 96, 4, 6, 2, 0, 8),         # odd k-step count per tap (cin 96 -> 3)
    (8, 64, 6, 3, 1, 0, 6),          # 8x8 grid (K = 64), two k-steps per tap
    (6, 32, 2, 4, 2, 2, 4),          # small grid, one k-step, a launch starting past block 0
])
def test_lic_latent_vs_torch(tmae, G, cin, nfr, nblk, nb, f_lo, f_hi):
    """tmae_lic_latent (the latent partial sums of every stack's first conv, mcm.py _slices) against torch's fp32
    conv2d of the same bf16-rounded operands: every block of the packing one stack, problem j reading its own
    input and the blocks from f_off[j]; columns outside the launch's fragments untouched"""
    from textmae_amd import ops

    torch.manual_seed(G * 1000 + cin)
    n = 5
    rows = n * G * G
    ldx = cin + 32
    xs = [_bf(torch.randn(rows, ldx, device=DEV)) for _ in range(nb)]
    co = 16 * nfr
    ws = [_bf(torch.randn(co, cin + 16, 3, 3, device=DEV) / (9 * cin) ** 0.5) for _ in range(nblk)]
    wpk = torch.stack([ops.pack_lic_stack_weight(w[:, :cin]) for w in ws]).contiguous()
    per = nblk // nb  # blocks per problem
    f_off = [j * per * nfr for j in range(nb)]
    ldy = nblk * co + 8
    y = torch.full((rows, ldy), float("nan"), device=DEV)
    ops.lic_latent(n, G, [x.to(torch.bfloat16) for x in xs], ldx, cin, wpk, nfr, wpk[0].numel(), f_off, f_lo, f_hi,
                   y, ldy)
    torch.cuda.synchronize()
    err = 0.0
    for j in range(nb):
        h = xs[j][:, :cin].reshape(n, G, G, cin).permute(0, 3, 1, 2)
        f = f_off[j] + f_lo
        while f < f_off[j] + f_hi:
            b, fi = divmod(f, nfr)
            nf = min(nfr - fi, f_off[j] + f_hi - f)
            ref = F.conv2d(h, ws[b][16 * fi:16 * (fi + nf), :cin], padding=1).permute(0, 2, 3, 1).reshape(rows, -1)
            got = y[:, 16 * f:16 * (f + nf)]
            err = max(err, _maxrel(got, ref))
            f += nf
    check("lic_latent_maxrel", err, LATENT_MAXREL)
    # columns of the fragments outside [f_lo, f_hi) of every problem keep their NaN
    mask = torch.ones(ldy, dtype=torch.bool, device=DEV)
    for j in range(nb):
        mask[16 * (f_off[j] + f_lo):16 * (f_off[j] + f_hi)] = False
    assert torch.isnan(y[:, mask]).all()


@pytest.mark.parametrize("G,cin,cout,nb,act", [(12, 384, 336, 1, True), (12, 384, 384, 2, False), (8, 96, 48, 2, True)])
def test_lic_latent_bias_act_bf16(tmae, G, cin, cout, nb, act):
    """the resident-input conv as h_a's first layers / h_s's last (mcm.py): bias, GELU, bf16 output at per-problem
    offsets, an odd fragment count (336 = 21 fragments: the last wave's lone fragment) -- against torch's fp32 conv2d
    + bias (+ GELU) of the same bf16 operands"""
    from textmae_amd import ops

    torch.manual_seed(cin + cout + nb)
    n = 4
    rows = n * G * G
    xs = [_bf(torch.randn(rows, cin, device=DEV)) for _ in range(nb)]
    ws = [_bf(torch.randn(cout, cin, 3, 3, device=DEV) / (9 * cin) ** 0.5) for _ in range(nb)]
    bs = [torch.randn(cout, device=DEV) for _ in range(nb)]
    nfr = -(-cout // 16)
    wpk = torch.stack([ops.pack_lic_stack_weight(w) for w in ws]).contiguous()
    y = torch.full((nb, rows, cout), float("nan"), device=DEV).to(torch.bfloat16)
    ops.lic_latent(n, G, [x.to(torch.bfloat16) for x in xs], cin, cin, wpk, nfr, wpk[0].numel(),
                   [j * nfr for j in range(nb)], 0, nfr, y, cout, y_s=[j * rows * cout for j in range(nb)], biases=bs,
                   act=ops.ACT_GELU if act else ops.ACT_NONE, y_bf16=True)
    torch.cuda.synchronize()
    err = 0.0
    for j in range(nb):
        h = xs[j].view(n, G, G, cin).permute(0, 3, 1, 2)
        ref = F.conv2d(h, ws[j], bs[j], padding=1).permute(0, 2, 3, 1).reshape(rows, cout)
        if act:
            ref = F.gelu(ref)
        err = max(err, _maxrel(y[j].float(), ref))
    check("lds_conv_maxrel", err, STACK_MAXREL)


def _gelu_grad(x):
    return 0.5 * (1.0 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5


@pytest.mark.parametrize("G,P,routed", [(12, 2, False), (12, 3, False), (8, 1, False), (12, 2, True), (8, 1, True),
                                        (12, 3, True)])
def test_lic_stack_bwd_vs_torch(tmae, G, P, routed):
    """TMAE_LIC_STACK_BWD (the fused data-gradient chain of a stack's layers 4..1, mcm_train._fused_dgrads) against
    torch: per layer dx = conv_transpose2d(d, W) (conv2d's input gradient) * GELU'(pre), rounded to bf16 as the
    kernel keeps it in LDS; every layer's output compared (the weight gradients' operands)"""
    from textmae_amd import ops

    torch.manual_seed(7 + G + P)
    n = 3
    rows = n * G * G
    chans = [224] + MID  # forward layer l: chans[l] -> chans[l + 1]; the backward runs 4..1
    ws = [[_bf(torch.randn(chans[l + 1], chans[l], 3, 3, device=DEV) / (9 * chans[l]) ** 0.5) for l in range(5)]
          for _ in range(P)]
    pres = {l: _bf(torch.randn(P, rows, chans[l + 1], device=DEV)) for l in range(4)}  # GELU inputs of layers 0..3
    dtop = _bf(torch.randn(P, rows, chans[5], device=DEV))
    wpk = [torch.stack([ops.pack_lic_stack_weight_t(ws[p][l]) for p in range(P)]).contiguous() for l in (4, 3, 2, 1)]
    outs = [torch.full((P, rows, chans[l + 1]), float("nan"), device=DEV).to(torch.bfloat16) for l in (3, 2, 1, 0)]
    st = {"x1": (rows * chans[5], 0)}
    for k, l in enumerate((3, 2, 1, 0)):
        st[f"w{k}"] = (wpk[k][0].numel(), 0)
        st[f"s{k}"] = (rows * chans[l + 1], 0)
    couts = [chans[l + 1] for l in (3, 2, 1, 0)]
    routes = None
    cin0, split = 96 + 384, (384, 64, 32)  # the first conv's input: latent | support | own slot, as three ranges
    if routed:  # + the first conv's input gradient, added into per-problem f32 accumulators (prior contents kept)
        w0 = [_bf(torch.randn(chans[1], cin0, 3, 3, device=DEV) / (9 * cin0) ** 0.5) for _ in range(P)]
        wpk.append(torch.stack([ops.pack_lic_stack_weight_t(w) for w in w0]).contiguous())
        st["w4"] = (wpk[4][0].numel(), 0)
        couts.append(cin0)
        # each range's accumulators of all problems at one constant stride inside one buffer (the route stride
        # lic_stack_bwd derives from problems 0 -> 1 must hold for every later problem too: P = 3 checks it)
        bufs = [torch.randn(P, rows, c + 8, device=DEV) for c in split]
        accs = [[b[p] for b in bufs] for p in range(P)]
        acc0 = [[a.clone() for a in ap] for ap in accs]
        routes = [[(a, c + 8, c) for a, c in zip(ap, split)] for ap in accs]
    ops.lic_stack_bwd(n, G, dtop.to(torch.bfloat16), chans[5], chans[5], wpk, couts,
                      [pres[l].to(torch.bfloat16) for l in (3, 2, 1, 0)], outs, nb=(P, 1), strides=st, routes=routes)
    torch.cuda.synchronize()
    err = 0.0
    for p in range(P):
        d = dtop[p]
        for k, l in enumerate((3, 2, 1, 0)):  # forward layer l + 1's input gradient -> layer l's pre-activation gradient
            w = ws[p][l + 1]
            h = d.view(n, G, G, -1).permute(0, 3, 1, 2)
            dx = F.conv_transpose2d(h, w, padding=1).permute(0, 2, 3, 1).reshape(rows, -1)
            ref = dx * _gelu_grad(pres[l][p])
            err = max(err, _maxrel(outs[k][p].float(), ref))
            d = _bf(ref)
        if routed:  # d = layer 0's pre-activation gradient (bf16): the first conv's input gradient, routed
            h = d.view(n, G, G, -1).permute(0, 3, 1, 2)
            dx = F.conv_transpose2d(h, w0[p], padding=1).permute(0, 2, 3, 1).reshape(rows, -1)
            c0 = 0
            for a, a0, c in zip(accs[p], acc0[p], split):
                err = max(err, _maxrel(a[:, :c] - a0[:, :c], dx[:, c0:c0 + c]))
                assert torch.equal(a[:, c:], a0[:, c:])  # the row padding untouched
                c0 += c
    check("lic_stack_bwd_maxrel", err, STACK_MAXREL)


def test_lic_stack_rejects_oversized(tmae):
    from textmae_amd import ops

    x = torch.zeros(144, 256, dtype=torch.bfloat16, device=DEV)
    w = [torch.zeros(1, dtype=torch.bfloat16, device=DEV)] * 5
    b = [torch.zeros(256, device=DEV)] * 5
    y = torch.zeros(144, 32, device=DEV)
    with pytest.raises(ValueError, match="input channels"):
        ops.lic_stack(1, 12, x, 256, 256, w, b, MID, y, 32, True)
    with pytest.raises(ValueError, match="grid"):
        ops.lic_stack(1, 13, x, 32, 256, w, b, MID, y, 32, True)


def test_mcm_fused_stacks_match_layerwise(tmae):
    """MCM eval forward, bf16, ViT-B 256^2 K=144 at batch 8: fused slice stacks vs the per-layer launches"""
    torch.manual_seed(3)
    m = tmae.MCM(img_size=256, num_keep_patches=144).to(DEV).eval()
    m.compute_dtype = torch.bfloat16
    m.distortion = "none"
    imgs = torch.randn(8, 3, 256, 256, device=DEV)
    scores = torch.rand(8, 256, device=DEV)
    outs = {}
    from textmae_amd import mcm as mcm_mod

    ex_cls = mcm_mod._Executor
    try:
        ex_cls.USE_LIC_CHAIN = False  # MUSIG holds the batched slices' mu / sigma only without the chain
        for flag in ("1", "0"):
            ex_cls.USE_LIC_STACK = flag == "1"
            m._exec = None
            with torch.no_grad():
                o = m(imgs, scores)
            assert (m._exec.lstk is not None) == (flag == "1")
            ex = m._exec
            # MUSIG holds mu / sigma of the batched slices 6..11; YH - YPRE = 0.5 tanh(lrp) of every slice
            outs[flag] = {"x_hat": o["x_hat"].clone(), "y": o["likelihoods"]["y"].clone(),
                          "yh": ex.YH.float().clone(), "musig": ex.MUSIG.clone(),
                          "lrp": (ex.YH.float() - ex.YPRE).clone()}
    finally:
        ex_cls.USE_LIC_STACK = True
        ex_cls.USE_LIC_CHAIN = True
        m._exec = None
    a, b = outs["1"], outs["0"]
    flips = int(((a["yh"] - b["yh"]).abs() > 0.5).sum())
    xr = float((a["x_hat"] - b["x_hat"]).norm() / b["x_hat"].norm())
    ly = (a["y"].double().log() - b["y"].double().log()).abs()
    print(f"fused vs layerwise: y_hat flips {flips} of {a['yh'].numel()}, x_hat rel L2 {xr:.2e}, "
          f"log y-lik max diff {float(ly.max()):.2e} mean {float(ly.mean()):.2e}")
    e_ms, e_lrp = _maxrel(a["musig"], b["musig"]), _maxrel(a["lrp"], b["lrp"])
    print(f"  mu/sigma (slices 6..11) max rel {e_ms:.2e}; 0.5 tanh(lrp) max rel {e_lrp:.2e}")
    record("log_ylik_maxdiff", float(ly.max()))
    # bounds about 2x the measured values (5.4e-4, 1.0e-2, 0 flips, 3.0e-3, 0)
    check("musig_maxrel", e_ms, 1.5e-3)
    check("lrp_maxrel", e_lrp, 2e-2)
    check("y_hat_flip_frac", flips / a["yh"].numel(), 1e-4, strict=False)
    check("x_hat_relL2", xr, 6e-3)
    check("log_ylik_meandiff", float(ly.mean()), 1e-3)


@pytest.mark.parametrize("training", [False, True])
def test_mcm_chained_slices_bitwise(tmae, training):
    """serial slices chained (mean stack -> y_hat_pre -> lrp stack in one launch, likelihoods deferred) against
    the separate mean/scale, Gaussian and lrp launches: the same arithmetic in the same order, so x_hat, both
    likelihoods and y_hat are bitwise equal (eval, and train-mode quantisation noise injected)"""
    from textmae_amd import mcm as mcm_mod

    torch.manual_seed(4)
    m = tmae.MCM(img_size=256, num_keep_patches=144).to(DEV).eval()
    m.compute_dtype = torch.bfloat16
    m.distortion = "none"
    imgs = torch.randn(6, 3, 256, 256, device=DEV)
    scores = torch.rand(6, 256, device=DEV)
    noise = (torch.rand(6, 192, 3, 3, device=DEV) - 0.5, torch.rand(6, 384, 12, 12, device=DEV) - 0.5)
    outs = {}
    ex_cls = mcm_mod._Executor
    try:
        for flag in ("1", "0"):
            ex_cls.USE_LIC_CHAIN = flag == "1"
            m._exec = None
            m.train(training)
            with torch.no_grad():
                o = m(imgs, scores, noise=noise) if training else m(imgs, scores)
            outs[flag] = (o["x_hat"].clone(), o["likelihoods"]["y"].clone(), o["likelihoods"]["z"].clone(),
                          m._exec.YH.clone())
    finally:
        ex_cls.USE_LIC_CHAIN = True
        m._exec = None
        m.eval()
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a, b)
