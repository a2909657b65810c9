"""Per-kernel parity: each HIP kernel vs a plain PyTorch fp32 CPU reference of the same op (or the
oracle, for the masking and entropy models).  Tolerances: f32 MFMA path 1e-4 relative (it is an exact
f32 fma chain; differences are summation order only), bf16 path 7e-3 relative (operand rounding);
integer outputs bit-exact."""
import os

import numpy as np
import pytest
import torch
from parity_log import check  # noqa: E402
import torch.nn.functional as F

from oracle import ids as ids_oracle
from oracle import mcm_oracle as orc

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def tol(dtype):
    # bf16: about 2x the largest error measured over these cases (3.3e-3, LayerNorm D=512;
    # profiles/r03/parity_metrics.jsonl)
    return 1e-4 if dtype == torch.float32 else 7e-3


DTYPES = [torch.float32, torch.bfloat16]


# ------------------------------------------------------------------------------------ masking
def test_ids_kernel_bit_exact_vs_reference_golden(golden_dir, tmae):
    d = np.load(os.path.join(golden_dir, "ids_shuffle.npz"))
    for k in sorted(d.files):
        if not k.endswith("_scores"):
            continue
        key = k[: -len("_scores")]
        K = int(key.split("_")[1][1:])
        s = torch.from_numpy(d[k]).to(DEV)
        shuf, rest = tmae.ops.ids_shuffle(s, K)
        expect = d[key + "_ids"].astype(np.int64)
        assert np.array_equal(shuf.cpu().numpy(), expect), key
        assert np.array_equal(rest.cpu().numpy(), np.argsort(expect, axis=1)), key


@pytest.mark.parametrize("L,K", [(256, 144), (196, 64), (1024, 400), (1, 1), (100, 0)])
def test_ids_kernel_vs_oracle_random(tmae, L, K):
    rng = np.random.default_rng(L + K)
    s = np.concatenate([rng.random((64, L), dtype=np.float32),
                        (rng.integers(0, 5, (64, L)) * rng.integers(1, 4, (64, L))).astype(np.float32) / 12.0])
    shuf, rest = tmae.ops.ids_shuffle(torch.from_numpy(s).to(DEV), K)
    es, er = ids_oracle.ids_shuffle(s, K)
    assert np.array_equal(shuf.cpu().numpy(), es)
    assert np.array_equal(rest.cpu().numpy(), er)


def test_ids_kernel_rejects_k_gt_l(tmae):
    with pytest.raises(ValueError, match="Number of patches"):
        tmae.ops.ids_shuffle(torch.zeros(2, 16, device=DEV), 17)


# ------------------------------------------------------------------------------------ transformer pieces
@pytest.mark.parametrize("D", [768, 512, 64, 1024])
@pytest.mark.parametrize("dtype", DTYPES)
def test_layernorm(tmae, D, dtype):
    torch.manual_seed(D)
    x = torch.randn(3, 37, D) * 3 + 1
    w, b = torch.randn(D), torch.randn(D)
    # drop row 0 of every group of 37 (the cls-dropping remap)
    y = tmae.ops.layernorm(x.to(DEV), w.to(DEV), b.to(DEV), 1e-6, dtype, rows=3 * 36, row_group=36,
                           group_stride=37, row_offset=1)
    ref = F.layer_norm(x[:, 1:], (D,), w, b, 1e-6).reshape(-1, D)
    check("rel:y_float", rel(y.float(), ref), tol(dtype))


# bench-sized row counts, ragged against the 4-row block
@pytest.mark.parametrize("groups,glen,D", [(3, 2731, 768), (5, 1700, 1024), (5, 1700, 512), (3, 2731, 2048)])
def test_layernorm_multirow(tmae, groups, glen, D):
    torch.manual_seed(glen + D)
    x = torch.randn(groups, glen, D) * 2 - 1
    w, b = torch.randn(D), torch.randn(D)
    y = tmae.ops.layernorm(x.to(DEV), w.to(DEV), b.to(DEV), 1e-6, torch.float32, rows=groups * (glen - 1),
                           row_group=glen - 1, group_stride=glen, row_offset=1)
    ref = F.layer_norm(x[:, 1:], (D,), w, b, 1e-6).reshape(-1, D)
    assert (y.cpu() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("M,N,K", [(9280, 2304, 768), (300, 64, 32), (129, 704, 640), (77, 32, 96), (1, 4, 8)])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("act", [0, 1])
def test_linear(tmae, M, N, K, dtype, act):
    torch.manual_seed(M + N + K)
    x, w, b = torch.randn(M, K), torch.randn(N, K) / K ** 0.5, torch.randn(N)
    y = tmae.ops.linear(x.to(DEV).to(dtype), w.to(DEV).to(dtype), b.to(DEV), dtype, act=act)
    ref = F.linear(x.to(dtype).float(), w.to(dtype).float(), b)
    if act:
        ref = F.gelu(ref)
    check("rel:y_float", rel(y.float(), ref), tol(dtype))


@pytest.mark.parametrize("dtype", DTYPES)
def test_linear_f32_source_and_residual(tmae, dtype):
    torch.manual_seed(3)
    M, N, K = 500, 384, 512
    x, w, b = torch.randn(M, K), torch.randn(N, K) / K ** 0.5, torch.randn(N)
    y = tmae.ops.linear(x.to(DEV), w.to(DEV).to(dtype), b.to(DEV), dtype, out_dtype=torch.float32)
    check("rel:y", rel(y, F.linear(x.to(dtype).float(), w.to(dtype).float(), b)), tol(dtype))
    r0 = torch.randn(M, N)
    r = r0.to(DEV).clone()
    tmae.ops.linear_residual(x.to(DEV).to(dtype), w.to(DEV).to(dtype), b.to(DEV), r, dtype)
    check("rel:r", rel(r, r0 + F.linear(x.to(dtype).float(), w.to(dtype).float(), b)), tol(dtype))


def _ref_attn(qkv, B, T, H, dh):
    q, k, v = qkv.reshape(B, T, 3, H, dh).permute(2, 0, 3, 1, 4)
    a = ((q @ k.transpose(-2, -1)) * dh ** -0.5).softmax(-1)
    return (a @ v).transpose(1, 2).reshape(B * T, H * dh)


@pytest.mark.parametrize("B,T,H,dh", [(4, 145, 12, 64), (3, 257, 16, 32), (2, 17, 2, 32), (1, 32, 1, 64),
                                      (2, 33, 4, 64), (2, 65, 16, 80), (1, 161, 3, 80)])
@pytest.mark.parametrize("dtype", DTYPES)
def test_mha(tmae, B, T, H, dh, dtype):
    torch.manual_seed(T)
    qkv = torch.randn(B * T, 3 * H * dh) * 1.5
    out = tmae.ops.mha(qkv.to(dtype).to(DEV), B, T, H, dh, dh ** -0.5, dtype)
    check("rel:out_float", rel(out.float(), _ref_attn(qkv.to(dtype).float(), B, T, H, dh)), (1e-4 if dtype == torch.float32 else 7e-3))


@pytest.mark.parametrize("B,T,H,dh", [(64, 145, 12, 64), (64, 257, 16, 32), (64, 65, 12, 64), (3, 145, 12, 64),
                                      (2, 257, 16, 32), (1, 129, 2, 64), (2, 288, 4, 32), (2, 160, 1, 64)])
def test_qkv_attn_fused_bitwise(tmae, B, T, H, dh):
    """tmae_qkv_attn_fwd (qkv Linear + attention in one launch, Q / K / V kept in LDS) equals the unfused
    tmae_linear_fwd(qkv) + tmae_mha_fwd bit for bit (same MFMA accumulation order, same bias rounding, same
    attention core), and both are within the bf16 bound of the fp32 reference"""
    if not tmae.ops.qkv_attn_supported(T, H, dh, torch.bfloat16):
        pytest.skip("no fused kernel for this shape")
    torch.manual_seed(T + H)
    D = H * dh
    x = (torch.randn(B * T, D) * 1.5).to(torch.bfloat16).to(DEV)
    w = (torch.randn(3 * D, D) / D ** 0.5).to(torch.bfloat16).to(DEV)
    b = (torch.randn(3 * D) * 0.1).to(DEV)
    scale = dh ** -0.5
    qkv = tmae.ops.linear(x, w, b, torch.bfloat16)
    ref = tmae.ops.mha(qkv, B, T, H, dh, scale, torch.bfloat16)
    out = torch.full((B * T, D), float("nan"), dtype=torch.bfloat16, device=DEV)
    tmae.ops.qkv_attn(x, w, b, B, T, H, dh, scale, torch.bfloat16, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, ref), float((out.float() - ref.float()).abs().max())
    if B <= 3:
        r32 = _ref_attn((x.float() @ w.float().t() + b).cpu(), B, T, H, dh)
        check("rel:out_float", rel(out.float(), r32), 1.5e-2)


# ------------------------------------------------------------------------------------ convs
def _nhwc(x, dtype):
    return x.permute(0, 2, 3, 1).contiguous().to(dtype).to(DEV)


def _wk(w, dtype):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous().to(dtype).to(DEV)


@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("H", [12, 3, 7])
def test_conv3x3_two_segments(tmae, stride, dtype, H):
    torch.manual_seed(stride + H)
    n, c1, c2, cout = 3, 40, 24, 48
    xa, xb = torch.randn(n, c1, H, H), torch.randn(n, c2, H, H)
    w, b = torch.randn(cout, c1 + c2, 3, 3) / (9 * (c1 + c2)) ** 0.5, torch.randn(cout)
    ref = F.gelu(F.conv2d(torch.cat([xa, xb], 1).to(dtype).float(), w.to(dtype).float(), b, stride=stride,
                          padding=1))
    Ho = ref.shape[2]
    # segment 2 lives inside a wider NHWC buffer (channel offset + stride)
    wide = torch.zeros(n, H, H, c2 + 16)
    wide[..., 8:8 + c2] = xb.permute(0, 2, 3, 1)
    wide = wide.to(dtype).to(DEV)
    y = torch.empty(n * Ho * Ho, cout, device=DEV)
    tmae.ops.conv3x3(_nhwc(xa, dtype), c1, c1, n, H, H, _wk(w, dtype), b.to(DEV), y, cout, cout, dtype,
                     stride=stride, act=1, x2=wide.data_ptr() + 8 * wide.element_size(), c2=c2, ld2=c2 + 16)
    check("rel:y_view_n_Ho_Ho_cout_permute_0_3_1_2", rel(y.view(n, Ho, Ho, cout).permute(0, 3, 1, 2), ref), tol(dtype))


@pytest.mark.parametrize("cin,c2,H,stride,cout,ps", [(336, 0, 12, 2, 288, False), (288, 0, 6, 1, 240, False),
                                                      (240, 0, 3, 1, 1152, True), (160, 32, 7, 2, 96, False),
                                                      (136, 64, 6, 1, 64, True)])
def test_conv3x3_wide_k_iterator(tmae, cin, c2, H, stride, cout, ps):
    """bf16 implicit-GEMM convs of >= 128 input channels, which take the K-iterator source (gemm_core.h ConvSrcIt):
    the hyperprior's strided / 6x6 / 3x3 shapes, a pixel-shuffle epilogue, and two input segments whose boundary
    falls inside a 64-channel K-step (a chunk's tap and source change mid-sweep), against the fp32 conv2d"""
    torch.manual_seed(cin + H + stride)
    dt, n, c1 = torch.bfloat16, 4, cin - c2
    xa, xb = torch.randn(n, c1, H, H), torch.randn(n, max(c2, 1), H, H)
    w, b = torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(cout)
    x = torch.cat([xa, xb[:, :c2]], 1) if c2 else xa
    pre = F.conv2d(x.to(dt).float(), w.to(dt).float(), b, stride=stride, padding=1)
    ref = F.gelu(F.pixel_shuffle(pre, 2) if ps else pre)
    Ho = ref.shape[2]
    cy = cout // 4 if ps else cout
    y = torch.full((n * Ho * Ho, cy), float("nan"), device=DEV, dtype=dt)
    extra = dict(x2=_nhwc(xb, dt), c2=c2, ld2=c2) if c2 else {}
    tmae.ops.conv3x3(_nhwc(xa, dt), c1, c1, n, H, H, _wk(w, dt), b.to(DEV), y, cy, cout, dt, stride=stride, act=1,
                     pixel_shuffle=ps, **extra)
    torch.cuda.synchronize()
    assert not torch.isnan(y.float()).any()
    check(f"rel:wide_{cin}_{H}_{stride}_{ps}", rel(y.float().view(n, Ho, Ho, cy).permute(0, 3, 1, 2), ref), tol(dt))


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv3x3_batched_addend(tmae, dtype):
    """nb1 x nb2 problems in one launch, per-problem weights/bias/addend/outputs, shared input"""
    torch.manual_seed(11)
    n, H, cin, cout, nb1, nb2 = 2, 12, 64, 32, 2, 3
    x = torch.randn(n, cin, H, H)
    w = torch.randn(nb1, nb2, cout, cin, 3, 3) / (9 * cin) ** 0.5
    b = torch.randn(nb1, nb2, cout)
    add = torch.randn(n * H * H, 7 * cout)  # problem (b1, b2) reads columns (3*b1 + b2)*cout
    y = torch.empty(nb1, nb2, n * H * H, cout, device=DEV)
    wk = torch.stack([torch.stack([w[i, j].permute(0, 2, 3, 1).reshape(cout, -1) for j in range(nb2)])
                      for i in range(nb1)]).to(dtype).contiguous().to(DEV)
    tmae.ops.conv3x3(_nhwc(x, dtype), cin, cin, n, H, H, wk, b.to(DEV), y, cout, cout, dtype, act=1,
                     addend=add.to(DEV), ld_add=7 * cout, nb=(nb1, nb2),
                     strides={"w": (nb2 * cout * 9 * cin, cout * 9 * cin), "b": (nb2 * cout, cout),
                              "a": (3 * cout, cout), "y": (nb2 * n * H * H * cout, n * H * H * cout)})
    for i in range(nb1):
        for j in range(nb2):
            ref = F.conv2d(x.to(dtype).float(), w[i, j].to(dtype).float(), b[i, j], padding=1)
            ref = F.gelu(ref.permute(0, 2, 3, 1).reshape(-1, cout) + add[:, (3 * i + j) * cout:(3 * i + j + 1) * cout])
            check(f"rel:batched_{i}_{j}", rel(y[i, j], ref), tol(dtype))


@pytest.mark.parametrize("n", [5, 64])
def test_conv_halo_two_images(tmae, n):
    """the halo-staged conv (two images per workgroup) against the fp32 conv2d: odd batch (a half-empty last
    pair), two input segments, 2 problems with an addend, cin not a multiple of 64; every output written"""
    torch.manual_seed(n)
    H, c1, c2, cout, nb = 12, 160, 32, 224, 2
    xa = torch.randn(n * H * H, c1).to(torch.bfloat16)
    xb = torch.randn(n * H * H, c2).to(torch.bfloat16)
    w = (torch.randn(nb, cout, 9 * (c1 + c2)) / (9 * (c1 + c2)) ** 0.5).to(torch.bfloat16)
    b = torch.randn(nb, cout)
    add = torch.randn(n * H * H, 2 * cout)
    y = torch.full((nb, n * H * H, cout), float("nan"), device=DEV, dtype=torch.bfloat16)
    tmae.ops.conv3x3(xa.to(DEV), c1, c1, n, H, H, w.to(DEV), b.to(DEV), y, cout, cout, torch.bfloat16, act=1,
                     x2=xb.to(DEV), c2=c2, ld2=c2, addend=add.to(DEV), ld_add=2 * cout, nb=(1, nb),
                     strides={"w": (0, w[0].numel()), "b": (0, cout), "a": (0, cout), "y": (0, n * H * H * cout)})
    torch.cuda.synchronize()
    assert not torch.isnan(y.float()).any()
    x = torch.cat([xa, xb], 1).float().reshape(n, H, H, c1 + c2).permute(0, 3, 1, 2)
    for p in range(nb):
        wk = w[p].float().reshape(cout, 3, 3, c1 + c2).permute(0, 3, 1, 2)
        pre = F.conv2d(x, wk, b[p], padding=1).permute(0, 2, 3, 1).reshape(-1, cout) + add[:, p * cout:(p + 1) * cout]
        check("rel:y_float", rel(y[p].float(), F.gelu(pre)), 7e-3)


@pytest.mark.parametrize("dtype", DTYPES)
def test_conv3x3_lrp_epilogue(tmae, dtype):
    torch.manual_seed(12)
    n, H, cin, cout = 2, 12, 80, 32
    x = torch.randn(n, cin, H, H)
    w, b = torch.randn(cout, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(cout)
    src = torch.randn(n * H * H, 96) * 4
    ref = src[:, 40:72] + 0.5 * torch.tanh(
        F.conv2d(x.to(dtype).float(), w.to(dtype).float(), b, padding=1).permute(0, 2, 3, 1).reshape(-1, cout))
    y = torch.zeros(n * H * H, 96, dtype=dtype, device=DEV)
    y2 = torch.zeros(n * H * H, 64, dtype=dtype, device=DEV)
    s = src.to(DEV)
    es = y.element_size()
    tmae.ops.conv3x3(_nhwc(x, dtype), cin, cin, n, H, H, _wk(w, dtype), b.to(DEV), y.data_ptr() + 40 * es, 96, cout,
                     dtype, y_f32=(dtype == torch.float32), lrp_src=s.data_ptr() + 40 * 4, ld_src=96,
                     y2=y2.data_ptr() + 16 * es, ldy2=64)
    check("rel:y_40_72_float", rel(y[:, 40:72].float(), ref), tol(dtype))
    check("rel:y2_16_48_float", rel(y2[:, 16:48].float(), ref), tol(dtype))
    assert float(y[:, :40].abs().max()) == 0.0 and float(y[:, 72:].abs().max()) == 0.0


@pytest.mark.parametrize("dtype", DTYPES)
def test_subpel_conv(tmae, dtype):
    torch.manual_seed(5)
    n, H, cin, c = 2, 6, 48, 16
    x = torch.randn(n, cin, H, H)
    w, b = torch.randn(4 * c, cin, 3, 3) / (9 * cin) ** 0.5, torch.randn(4 * c)
    ref = F.gelu(F.pixel_shuffle(F.conv2d(x.to(dtype).float(), w.to(dtype).float(), b, padding=1), 2))
    y = torch.empty(n * 4 * H * H, c, device=DEV)
    tmae.ops.conv3x3(_nhwc(x, dtype), cin, cin, n, H, H, _wk(w, dtype), b.to(DEV), y, c, 4 * c, dtype,
                     act=1, pixel_shuffle=True)
    check("rel:y_view_n_2_H_2_H_c_permute_0_3_1_2", rel(y.view(n, 2 * H, 2 * H, c).permute(0, 3, 1, 2), ref), tol(dtype))


@pytest.mark.parametrize("training", [False, True])
@pytest.mark.parametrize("yt", DTYPES)
def test_gc_slices(tmae, training, yt):
    torch.manual_seed(21)
    n, HW, M, sw, nsl, yoff = 2, 16, 96, 16, 3, 32
    y = torch.randn(n * HW, M) * 5
    mu = torch.randn(2, nsl, n * HW, sw)
    sigma = torch.rand(nsl, n * HW, sw) * 3
    musig = torch.stack([mu[0], sigma])  # [mu | sigma] blocks like the executor's MUSIG
    noise = torch.rand(n, M, HW) - 0.5 if training else None
    lik = torch.zeros(n, M, HW, device=DEV)
    yh = torch.zeros(n * HW, M, dtype=yt, device=DEV)
    yh32 = torch.zeros(n * HW, M, device=DEV)
    ms = musig.to(DEV)
    tmae.ops.gc_slices(y.to(DEV), M, yoff, ms, ms.data_ptr() + nsl * n * HW * sw * 4, n * HW * sw, sw,
                       None if noise is None else noise.to(DEV), lik, M, yh, yt, M, yh32, M, n, HW, nsl, sw)
    for j in range(nsl):
        ch = slice(yoff + j * sw, yoff + (j + 1) * sw)
        ys = y[:, ch].reshape(n, HW, sw).permute(0, 2, 1)
        mj = mu[0, j].reshape(n, HW, sw).permute(0, 2, 1)
        sj = sigma[j].reshape(n, HW, sw).permute(0, 2, 1)
        nz = None if noise is None else noise[:, ch]
        ref = orc.gaussian_conditional(ys, sj, mj, nz)
        check("rel:lik_ch_cpu", rel(lik[:, ch].cpu(), ref), 1e-5)
        q = (torch.round(ys - mj) + mj).permute(0, 2, 1).reshape(-1, sw)
        assert torch.equal(yh32[:, ch].cpu(), q)
        assert rel(yh[:, ch].float(), q) <= (0 if yt == torch.float32 else 1e-2)


# ------------------------------------------------------------------------------------ entropy models
def _eb_module(tmae, C, seed):
    torch.manual_seed(seed)
    eb = tmae.EntropyBottleneck(C)
    with torch.no_grad():
        for n, p in eb.named_parameters():
            if "_factor" in n or "_matrix" in n:
                p.normal_(0, 0.5)
            if "quantiles" in n:
                p.add_(torch.rand_like(p) * 0.6 - 0.3)
    return eb


@pytest.mark.parametrize("training", [False, True])
def test_entropy_bottleneck(tmae, training):
    C = 192
    eb = _eb_module(tmae, C, 0)
    sd = {f"eb.{k}": v for k, v in eb.state_dict().items()}
    z = torch.randn(4, C, 3, 3) * 4
    noise = torch.rand(4, C, 3, 3) - 0.5 if training else None
    lik_ref, zhat_ref = orc.entropy_bottleneck(sd, "eb.", z, noise)
    eb = eb.to(DEV)
    out, lik = eb(z.to(DEV), training=training, noise=None if noise is None else noise.to(DEV))
    check("rel:lik", rel(lik, lik_ref), 1e-5)
    if not training:
        assert torch.equal(out.cpu(), zhat_ref)
    np.testing.assert_allclose(float(eb.loss().detach()), float(orc.eb_aux_loss(sd, "eb.")), rtol=1e-5)


@pytest.mark.parametrize("training", [False, True])
def test_gaussian_conditional(tmae, training):
    torch.manual_seed(2)
    y, mu = torch.randn(2, 32, 12, 12) * 5, torch.randn(2, 32, 12, 12)
    sigma = torch.rand(2, 32, 12, 12) * 3
    noise = torch.rand(2, 32, 12, 12) - 0.5 if training else None
    ref = orc.gaussian_conditional(y, sigma, mu, noise)
    gc = tmae.GaussianConditional(None).to(DEV)
    _, lik = gc(y.to(DEV), sigma.to(DEV), mu.to(DEV), training=training,
                noise=None if noise is None else noise.to(DEV))
    check("rel:lik", rel(lik, ref), 1e-5)


# ------------------------------------------------------------------------------------ embed / unembed
@pytest.mark.parametrize("dtype", DTYPES)
def test_patch_embed_kept_only(tmae, dtype):
    torch.manual_seed(9)
    n, img, P, D, K = 3, 64, 16, 128, 9
    L = (img // P) ** 2
    imgs = torch.rand(n, 3, img, img)
    w, b = torch.randn(D, 3, P, P) / (3 * P * P) ** 0.5, torch.randn(D)
    pos = torch.randn(1, L + 1, D)
    shuf = torch.stack([torch.randperm(L) for _ in range(n)])
    full = F.conv2d(imgs.to(dtype).float(), w.to(dtype).float(), b, stride=P).flatten(2).transpose(1, 2) + pos[:, 1:]
    ref = torch.gather(full, 1, shuf[:, :K].unsqueeze(-1).repeat(1, 1, D))
    tok = torch.zeros(n, K + 1, D, device=DEV)
    tmae.ops.patch_embed(imgs.to(DEV), shuf.to(DEV), w.view(D, -1).to(dtype).to(DEV), b.to(DEV), pos.to(DEV), tok,
                         K, P, dtype)
    check("rel:tok_1", rel(tok[:, 1:], ref), tol(dtype))


@pytest.mark.parametrize("ntok", [16, 17])
def test_decoder_embed_unshuffle(tmae, ntok):
    torch.manual_seed(ntok)
    n, L, Din, D = 2, 64, 96, 32
    x = torch.randn(n, ntok, Din)
    w, b = torch.randn(D, Din) / Din ** 0.5, torch.randn(D)
    pos, mask = torch.randn(1, L + 1, D), torch.randn(1, 1, D)
    shuf = torch.stack([torch.randperm(L) for _ in range(n)])
    rest = torch.argsort(shuf, 1)
    xd = F.linear(x, w, b)
    x_ = torch.cat([xd[:, 1:], mask.repeat(n, L + 1 - ntok, 1)], 1)
    x_ = torch.gather(x_, 1, rest.unsqueeze(-1).repeat(1, 1, D))
    ref = torch.cat([xd[:, :1], x_], 1) + pos
    out = torch.full((n, L + 1, D), float("nan"), device=DEV)
    s = shuf.to(DEV)
    tmae.ops.decoder_embed(x.reshape(-1, Din).to(DEV), w.to(DEV), b.to(DEV), pos.to(DEV), s, out, n, ntok, L,
                           torch.float32)
    tmae.ops.mask_rows(out, mask.to(DEV), pos.to(DEV), s, n, L, ntok, D)
    check("rel:out", rel(out, ref), 1e-5)


def test_decoder_pred_unpatchify(tmae):
    torch.manual_seed(4)
    n, L, Din, P = 2, 16, 64, 16
    x = torch.randn(n * L, Din)
    w, b = torch.randn(P * P * 3, Din) / 8, torch.randn(P * P * 3)
    ref = orc.unpatchify(F.linear(x, w, b).view(n, L, -1), P)
    imgs = torch.empty(n, 3, 64, 64, device=DEV)
    tmae.ops.decoder_pred(x.to(DEV), w.to(DEV), b.to(DEV), imgs, n, L, P, torch.float32)
    check("rel:imgs", rel(imgs, ref), 1e-5)


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("n,L,P,C", [(2, 16, 16, 3), (3, 256, 16, 3), (2, 4, 8, 1)])
def test_decoder_pred_channel_planar(tmae, dtype, n, L, P, C):
    """the channel-planar weight order (inference executor) gives the reference-order result bit for bit"""
    torch.manual_seed(L + P)
    Din = 64
    G = int(L ** 0.5)
    x = torch.randn(n * L, Din).to(dtype).to(DEV)
    w, b = (torch.randn(P * P * C, Din) / 8).to(dtype).to(DEV), torch.randn(P * P * C, device=DEV)
    ref = torch.empty(n, C, G * P, G * P, device=DEV)
    tmae.ops.decoder_pred(x, w, b, ref, n, L, P, dtype)
    perm = tmae.ops.pred_channel_planar_perm(P, C).to(DEV)
    out = torch.full_like(ref, float("nan"))
    tmae.ops.decoder_pred(x, w[perm].contiguous(), b[perm].contiguous(), out, n, L, P, dtype, channel_planar=True)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


@pytest.mark.parametrize("dtype", DTYPES)
def test_block_module(tmae, dtype):
    torch.manual_seed(0)
    blk = tmae.Block(128, 4, qkv_bias=True, norm_layer=lambda d: torch.nn.LayerNorm(d, eps=1e-6))
    x = torch.randn(3, 41, 128)
    sd = {f"b.{k}": v for k, v in blk.state_dict().items()}
    if dtype == torch.bfloat16:
        sd = {k: (v.to(dtype).float() if v.dim() == 2 else v) for k, v in sd.items()}
    ref = orc.block(x, sd, "b.", 4, 1e-6)
    blk = blk.to(DEV)
    blk.compute_dtype = dtype
    check("rel:blk_x_to_DEV", rel(blk(x.to(DEV)), ref), (1e-4 if dtype == torch.float32 else 7e-3))


# ------------------------------------------------------------------------------------ loader crops
def test_crop_normalize_u8_bitwise_torch(tmae):
    """the DIV2K-shaped loader sample (data.py): crop of a uint8 HWC image, ToTensor (/255) + Normalize,
    bitwise equal to the same torch f32 ops (utils/dataloader.py:58-61)"""
    g = torch.Generator().manual_seed(3)
    src = torch.randint(0, 256, (3, 61, 90, 3), dtype=torch.uint8, generator=g)
    S = 24
    crops = torch.tensor([[0, 0, 0], [2, 61 - S, 90 - S], [1, 17, 33], [2, 5, 0], [0, 37, 66]], dtype=torch.int32)
    mean, std = (0.485, 0.456, 0.406), (0.229, 0.224, 0.225)
    out = tmae.ops.crop_normalize_u8(src.to(DEV), crops.to(DEV), S, mean, std)
    m = torch.tensor(mean).view(3, 1, 1)
    s = torch.tensor(std).view(3, 1, 1)
    ref = torch.stack([(src[i, t:t + S, l:l + S].permute(2, 0, 1).float().div(255) - m) / s
                       for i, t, l in crops.tolist()])
    assert torch.equal(out.cpu(), ref)


def test_synthetic_crop_set_plan_is_seeded(tmae):
    from textmae_amd.data import SyntheticCropSet

    a = SyntheticCropSet(DEV, seed=5, rank=1, num_images=2, hw=(300, 400)).plan(3, 4)
    b = SyntheticCropSet(DEV, seed=5, rank=1, num_images=2, hw=(300, 400)).plan(3, 4)
    c = SyntheticCropSet(DEV, seed=5, rank=0, num_images=2, hw=(300, 400)).plan(3, 4)
    xa, sa = a.next()
    xb, sb = b.next()
    xc, _ = c.next()
    assert xa.shape == (4, 3, 256, 256) and sa.shape == (4, 256)
    assert torch.equal(xa, xb) and torch.equal(sa, sb) and not torch.equal(xa, xc)
