"""Benchmark: images/s of MCM encode + rate + decode (BASELINE.json metric) on MI355X.

One step = one MCM.forward (eval: masking ids on device, ViT-B/16 encoder, LIC hyperprior with
EntropyBottleneck + 12-slice GaussianConditional likelihoods, ViT decoder, unpatchify) over a batch
of 64 synthetic 256x256 RGB images with K=144 kept patches, bf16 MFMA operands (f32 accumulate,
f32 entropy models).  The forward is replayed as a HIP graph; inputs are resident in HBM.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...
    python bench.py --enc-dim 1024 --enc-depth 24 --enc-heads 16 --batch 128     # BASELINE config 4

Multi-GPU: images are independent, so every rank runs its own batch with no
collective on the data path ("weak" scaling); the barrier + max-over-ranks timing follows the
driver contract.  Rank 0 prints one JSON line.

Roofline (rank 0): one extra eager forward records every library launch with its kernel family and
algorithmic FLOPs; each family's launches are then replayed back to back between a HIP event pair on
the stream they run on, giving the family's kernel time per forward (DESIGN.md §5 lists the shape ->
family mapping; tools/family_summary.py gives the same split from a rocprofv3 kernel trace):
  * ``roofline`` = the family with the most kernel time (the dominant kernel), FLOPs / time;
  * ``roofline.attention_block`` = encoder / decoder (qkv GEMM + attention core + proj GEMM);
  * ``roofline.attention_core`` = the attention kernels alone (HBM/LDS-bound by AI, SURVEY (v)) where they run as
    their own launch; the bf16 forward fuses the qkv GEMM and the core into one launch (``qkv_attn_fused``).
"""
import argparse
import json
import os
import platform
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec encode+decode+rate, ViT-B 256×256 batch64, 1/2/4/8 MI355X"
PEAK_BF16 = 2.5e15               # MI355X_MICROARCH.md: dense bf16 MFMA
PEAK_HBM = 8.0e12
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--img", type=int, default=256)
    ap.add_argument("--keep", type=int, default=144)
    ap.add_argument("--enc-dim", type=int, default=768)
    ap.add_argument("--enc-depth", type=int, default=12)
    ap.add_argument("--enc-heads", type=int, default=12)
    ap.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=6.0, help="all-threads oracle sample length")
    ap.add_argument("--cpu-batch", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-leg", default=None, help=argparse.SUPPRESS)  # internal: one CPU-baseline leg
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--dump-launches", default=None, help="write every launch of one forward with its family and shape")
    ap.add_argument("--train-steps", type=int, default=10, help="training steps timed after the inference run")
    ap.add_argument("--train-warmup", type=int, default=3)
    ap.add_argument("--train-batch", type=int, default=64)
    ap.add_argument("--no-train", action="store_true")
    ap.add_argument("--mae-large", action="store_true",
                    help="add the literal BASELINE config 4 line (MAE ViT-L dec512d8b, batch 128, bf16)")
    ap.add_argument("--no-dp-rehearsal", dest="dp_rehearsal", action="store_false",
                    help="skip the one-rank RCCL GradSync overlap measurement at N=1")
    ap.add_argument("--no-distortion", dest="distortion_line", action="store_false",
                    help="skip the forward_loss (SSIM + L1 + VGG) line")
    ap.add_argument("--no-k64", dest="k64_line", action="store_false", help="skip the K=64 (config 2') line")
    ap.add_argument("--no-mae-train", dest="mae_train_line", action="store_false",
                    help="skip the MaskedAutoencoderViT training line")
    ap.add_argument("--kernel-reps", type=int, default=0, help="unused (kept for older command lines)")
    ap.add_argument("--backend", default="nccl", help="process-group backend (nccl = RCCL; gloo for a one-GPU rehearsal)")
    return ap.parse_args()


def vitb_default(args):
    """the BASELINE config 2 model (ViT-B encoder, K=144): the side lines run only next to it"""
    return args.keep == 144 and args.enc_dim == 768 and args.enc_depth == 12


def synthetic_inputs(batch, img, L, seed, device):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(batch, 3, img, img, generator=g)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 3, 1, 1)
    x = (x - mean) / std  # the train transform's Normalize (utils/dataloader.py:61)
    s = torch.rand(batch, L, generator=torch.Generator().manual_seed(seed + 1))
    return x.to(device), s.to(device)


# ------------------------------------------------------------------------------ algorithmic work
def gflop_per_image(m):
    """forward FLOPs per image by component (2 * MAC), from the constructor arithmetic MCM.py:77-354;
    counts what the reference computes (all L patches embedded, decoder_pred on L + 1 rows)"""
    E, Dd, M, N, S = m.encoder_embed_dim, m.decoder_embed_dim, m.latent_depth, m.hyperprior_depth, m.num_slices
    P, C = m.encoder_embed.patch_size[0], m.encoder_embed.proj.in_channels
    L, K = m.encoder_embed.num_patches, m.num_keep_patches
    g = int(round(K ** 0.5))
    f = {"patch_embed": 2 * L * E * C * P * P}

    def blocks(T, blks):
        gemm = core = 0
        for b in blks:
            D, h = b.attn.qkv.in_features, b.mlp.fc1.out_features
            gemm += 2 * T * D * (4 * D + 2 * h)
            core += 4 * T * T * D
        return gemm, core

    f["enc_gemm"], f["enc_core"] = blocks(K + 1, m.encoder_blocks)
    ga = [l for l in m.g_a if isinstance(l, torch.nn.Conv2d)]
    f["g_a"] = f["g_s"] = sum(2 * K * l.in_channels * l.out_channels for l in ga)
    tot, r = 0, g
    for l in m.h_a:
        if isinstance(l, torch.nn.Conv2d):
            ro = (r + 2 - 3) // l.stride[0] + 1
            tot += 2 * ro * ro * l.out_channels * l.in_channels * 9
            r = ro
    f["h_a"], hz = tot, r
    tot, r = 0, hz
    for l in m.h_s_mean:
        c = l if isinstance(l, torch.nn.Conv2d) else (l[0] if isinstance(l, torch.nn.Sequential) else None)
        if c is not None:
            tot += 2 * r * r * c.out_channels * c.in_channels * 9
            if c is not l:
                r *= 2
    f["h_s"] = 2 * tot

    def stack(seq):
        return sum(2 * K * c.in_channels * c.out_channels * 9 for c in seq if isinstance(c, torch.nn.Conv2d))

    f["cc"] = sum(stack(a) + stack(b) for a, b in zip(m.cc_transform_mean, m.cc_transform_scale))
    f["lrp"] = sum(stack(s) for s in m.lrp_transform)
    f["dec_embed"] = 2 * K * E * Dd
    f["dec_gemm"], f["dec_core"] = blocks(L + 1, m.decoder_blocks)
    f["dec_pred"] = 2 * (L + 1) * Dd * P * P * C
    return {k: v / 1e9 for k, v in f.items()}


# ------------------------------------------------------------------------------ per-launch timing
class LaunchTimer:
    """Records every launch of one eager forward through the library's call gate, tagged with its
    kernel family and algorithmic FLOPs, then replays each family's launches back to back on one
    stream (same arguments, same workspaces, in forward order) between a HIP event pair: the family's
    kernel time per forward without launch gaps or side-stream overlap -- the number a rocprofv3
    kernel trace sums for those kernels (cross-checked by tools/family_summary.py)."""

    def __init__(self, m, batch, reps=5):
        from textmae_amd import _lib

        self._lib = _lib
        self.m, self.B, self.reps = m, batch, reps
        self.E, self.Dd = m.encoder_embed_dim, m.decoder_embed_dim
        self.Te, self.Td = m.num_keep_patches + 1, m.encoder_embed.num_patches + 1
        self.calls = []
        self.conv_bytes = 0
        self.stack_bytes = 0
        self.hbm_bytes = {}  # memory-bound families: algorithmic HBM bytes per forward
        self.gemm_bytes = [0, 0]  # dense-source GEMM launches (PMC family "token_gemm"): [launches, algorithmic bytes]

    def _hbm(self, fam, nbytes):
        self.hbm_bytes[fam] = self.hbm_bytes.get(fam, 0) + nbytes

    def classify(self, name, a):
        B, E, Dd, Te, Td = self.B, self.E, self.Dd, self.Te, self.Td
        if name == "tmae_linear_fwd" or name == "tmae_linear_residual_fwd":
            M, N, K = (a[13], a[14], a[15]) if name == "tmae_linear_fwd" else (a[6], a[7], a[8])
            fl = 2.0 * M * N * K
            # algorithmic bytes: A + W + bias + the output (f32 residual: read and written)
            if name == "tmae_linear_fwd":
                es = 2 if a[17] == 1 else 4
                nb = M * K * (4 if a[1] else es) + N * K * es + N * 4 + M * N * (4 if a[9] else es) + \
                    (M * N * 4 if a[11] else 0)
            else:
                es = 2 if a[9] == 1 else 4
                nb = M * K * es + N * K * es + N * 4 + 2 * M * N * 4
            self.gemm_bytes[0] += 1
            self.gemm_bytes[1] += nb
            for side, D, T in (("enc", E, Te), ("dec", Dd, Td)):
                if M == B * T:
                    if name == "tmae_linear_fwd" and (N, K) == (3 * D, D):
                        return f"{side}_qkv", fl
                    if name == "tmae_linear_residual_fwd" and (N, K) == (D, D):
                        return f"{side}_proj", fl
                    if name == "tmae_linear_fwd" and K == D:
                        return f"{side}_fc1", fl
                    if name == "tmae_linear_residual_fwd":
                        return f"{side}_fc2", fl
            return "lic_1x1_gemm", fl
        if name == "tmae_qkv_attn_fwd":
            Bq, T, H, dh = a[4], a[5], a[6], a[7]
            D = H * dh
            fam = "enc_qkv_attn" if T == self.Te else "dec_qkv_attn"
            self._hbm(fam, Bq * T * D * 2 * 2 + 3 * D * D * 2 + 3 * D * 4)  # x in, O out (bf16), W, bias
            return fam, 2.0 * Bq * T * D * 3 * D + 4.0 * Bq * H * T * T * dh
        if name == "tmae_mha_fwd":
            Bq, T, H, dh = a[2], a[3], a[4], a[5]
            fam = "enc_attn_core" if T == Te else "dec_attn_core"
            es = 2 if a[7] == 1 else 4
            self._hbm(fam, Bq * T * H * dh * es * 4)  # qkv in (3 x), o out
            return fam, 4.0 * Bq * H * T * T * dh
        if name == "tmae_conv3x3":
            c = a[0]._obj
            Ho = (c.H + 2 - 3) // c.stride + 1
            Wo = (c.W + 2 - 3) // c.stride + 1
            nb, cin, es = c.nb1 * c.nb2, c.c1 + c.c2, (2 if a[1] == 1 else 4)
            # algorithmic bytes: input map + weights + output (+ partial-sum addend) of every problem
            self.conv_bytes += nb * (c.n * c.H * c.W * cin * es + c.cout * 9 * cin * es
                                     + c.n * Ho * Wo * c.cout * ((4 if c.y_f32 else 2) + (4 if c.addend else 0)))
            return "lic_conv3x3", 2.0 * nb * c.n * Ho * Wo * c.cout * 9 * cin
        if name == "tmae_lic_stack":
            c = a[0]._obj
            P, px = c.nb1 * c.nb2, c.n * c.G * c.G
            ch = [c.c1 + c.c2] + [c.cout[l] for l in range(c.nlayers)]
            fl = 2.0 * P * px * 9 * sum(ch[l] * ch[l + 1] for l in range(c.nlayers))
            # algorithmic bytes: layer-0 input, every layer's weights, the addend, the output (+ lrp source)
            self.stack_bytes += P * (px * ch[0] * 2 + sum(9 * ch[l] * ch[l + 1] * 2 for l in range(c.nlayers))
                                     + (px * ch[1] * 4 if c.addend else 0)
                                     + px * ch[-1] * ((4 if c.y_f32 else 2) + (4 if c.lrp_src else 0)))
            if c.flags & 1:  # chained: the mean problems (nb2 of them) go on with their lrp stacks
                c2 = [c.cc1 + c.ccout[c.cn - 1]] + [c.ccout[l] for l in range(c.cn)]
                fl += 2.0 * c.nb2 * px * 9 * sum(c2[l] * c2[l + 1] for l in range(c.cn))
                # support slots + y and mu in, y_hat_pre f32 out, lrp weights, addend, y_hat out (bf16)
                self.stack_bytes += c.nb2 * (px * c.cc1 * 2 + px * c2[-1] * (4 + 4 + 4 + 2)
                                             + sum(9 * c2[l] * c2[l + 1] * 2 for l in range(c.cn))
                                             + (px * c2[1] * 4 if c.cadd else 0))
            return "lic_stack", fl
        if name == "tmae_lic_latent":
            c = a[0]._obj
            px, ncol = c.n * c.G * c.G, 16 * (c.f_hi - c.f_lo)
            # algorithmic bytes: each problem's input map, its weight fragments, the f32 output columns
            self.conv_bytes += c.nb * (px * c.cin * 2 + ncol * 9 * c.cin * 2 + px * ncol * 4)
            return "lic_latent", 2.0 * c.nb * px * ncol * 9 * c.cin
        if name == "tmae_patch_embed_fwd":
            return "patch_embed", 2.0 * a[6] * a[13] * a[11] * a[7] * a[10] * a[10]
        if name == "tmae_patch_embed_gathered":  # (patches, ids, w, b, pos, tok, n, Kw, D, L, keep, ...)
            es = 2 if a[11] == 1 else 4
            self.gemm_bytes[0] += 1
            self.gemm_bytes[1] += a[6] * a[10] * a[7] * es + a[8] * a[7] * es + a[6] * a[10] * a[8] * 4
            return "patch_embed", 2.0 * a[6] * a[10] * a[8] * a[7]
        if name == "tmae_patch_gather":  # the kept-patch gather in front of it (time only)
            return "patch_embed", 0.0
        if name == "tmae_decoder_embed_fwd":  # (x, x_f32, w, b, pos, ids, out, n, ntok, L, Din, D, dtype, ...)
            es = 2 if a[12] == 1 else 4
            self.gemm_bytes[0] += 1
            self.gemm_bytes[1] += a[7] * a[8] * a[10] * (4 if a[1] else es) + a[11] * a[10] * es + a[7] * a[8] * a[11] * 4
            return "dec_embed", 2.0 * a[7] * a[8] * a[10] * a[11]
        if name in ("tmae_decoder_pred_fwd", "tmae_decoder_pred_cp_fwd"):  # (x, w, b, imgs, n, L, Din, C, H, W, P, dt)
            es = 2 if a[11] == 1 else 4
            npix = a[7] * a[10] * a[10]
            self.gemm_bytes[0] += 1
            self.gemm_bytes[1] += a[4] * a[5] * a[6] * es + npix * a[6] * es + a[4] * a[5] * npix * 4
            return "dec_pred", 2.0 * a[4] * a[5] * a[6] * a[7] * a[10] * a[10]
        if name == "tmae_layernorm_fwd":
            rows, D = a[4], a[5]
            self._hbm("layernorm", rows * D * (4 + (2 if a[10] == 1 else 4)) + 2 * D * 4)  # x f32 in, y out, gamma/beta
            return "layernorm", 0.0
        if name == "tmae_gc_slices_fwd":
            # y, mu, sigma in, likelihood out (f32), y_hat_pre out (operand dtype) and its f32 copy, noise in
            n_el = a[15] * a[16] * a[17] * a[18]
            per = 16 + ((2 if a[11] == 1 else 4) if a[10] else 0) + (4 if a[13] else 0) + (4 if a[7] else 0)
            self._hbm("gc_slices", n_el * per)
            return "gc_slices", 0.0
        if name == "tmae_eb_likelihood_fwd":
            n_el = a[7] * a[8] * a[9]  # z in, likelihood out (f32), z_hat out, noise in
            self._hbm("eb_likelihood", n_el * (8 + ((2 if a[5] == 1 else 4) if a[4] else 0) + (4 if a[2] else 0)))
            return "eb_likelihood", 0.0
        return "other:" + name, 0.0

    def describe(self, name, a):
        """the shape a launch was classified on (the shape -> family mapping, written out by --dump-launches)"""
        if name == "tmae_linear_fwd":
            return {"M": a[13], "N": a[14], "K": a[15]}
        if name == "tmae_linear_residual_fwd":
            return {"M": a[6], "N": a[7], "K": a[8]}
        if name == "tmae_mha_fwd":
            return {"B": a[2], "T": a[3], "H": a[4], "dh": a[5]}
        if name == "tmae_lic_stack":
            c = a[0]._obj
            return {"n": c.n, "G": c.G, "cin": c.c1 + c.c2, "couts": [c.cout[l] for l in range(c.nlayers)],
                    "problems": c.nb1 * c.nb2, "addend": bool(c.addend), "lrp": bool(c.lrp_src)}
        if name == "tmae_conv3x3":
            c = a[0]._obj
            return {"n": c.n, "H": c.H, "W": c.W, "cin": c.c1 + c.c2, "cout": c.cout, "problems": c.nb1 * c.nb2,
                    "stride": c.stride, "out_f32": bool(c.y_f32), "addend": bool(c.addend)}
        return {}

    def run(self, fn, live=("lic_stack",)):
        """classify every library launch of fn() (one eager forward); the launches of the `live` families are also
        bracketed by HIP events on the stream they are launched on, so their duration INSIDE the forward (beside the
        side stream's kernels, as in the graphed step) is measured live (self.live_us: family -> mean us)"""
        orig = self._lib.call
        calls = self.calls
        evs = {}

        def record(name, *args):
            fam, fl = self.classify(name, args)
            calls.append((fam, fl, name, args))
            if fam not in live:
                return orig(name, *args)
            st_ = torch.cuda.ExternalStream(args[-1]) if args[-1] else torch.cuda.current_stream()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st_)
            r = orig(name, *args)
            b.record(st_)
            evs.setdefault(fam, []).append((a, b))
            return r

        self._lib.call = record
        try:
            fn()
        finally:
            self._lib.call = orig
        torch.cuda.synchronize()
        self.live_us = {f: 1e3 * sum(a.elapsed_time(b) for a, b in v) / len(v) for f, v in evs.items()}
        fams = {}
        for fam, fl, name, args in calls:
            t = fams.setdefault(fam, [[], 0.0])
            t[0].append((name, args))
            t[1] += fl
        out = {}
        st = torch.cuda.current_stream()
        try:
            torch._C._cuda_sleep(1000)  # a marker kernel in a rocprofv3 trace: the replays follow it
        except Exception:
            pass
        for fam, (launches, fl) in fams.items():
            if fl <= 0 and fam not in self.hbm_bytes:
                continue  # ids / copies / state-carrying entropy-model steps: not replayed
            launches = [(name, args[:-1] + (st.cuda_stream,)) for name, args in launches]  # stream is the last arg
            for name, args in launches:  # warm
                orig(name, *args)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(self.reps):
                for name, args in launches:
                    orig(name, *args)
            e1.record(st)
            e1.synchronize()
            out[fam] = [len(launches), e0.elapsed_time(e1) * 1e-3 / self.reps, fl]
        return out


def roofline_report(m, imgs, scores, batch, dump=None, profiled=True):
    lt = LaunchTimer(m, batch)
    with torch.no_grad():
        fam = lt.run(lambda: m(imgs, scores))
    if dump:
        rows = [{"i": i, "entry": name, "family": f, "gflop": round(fl / 1e9, 4), "shape": lt.describe(name, args)}
                for i, (f, fl, name, args) in enumerate(lt.calls)]
        with open(dump, "w") as fh:
            json.dump({"batch": batch, "launches": rows}, fh, indent=0)
    mf = {k: v for k, v in fam.items() if v[2] > 0}
    agg = {"token_gemm": [k for k in mf if k.split("_")[-1] in ("qkv", "proj", "fc1", "fc2")],
           "token_gemm_with_qkv_attn": [k for k in mf if k.split("_")[-1] in ("qkv", "proj", "fc1", "fc2")
                                        or k.endswith("qkv_attn")],
           "lic_conv3x3": ["lic_conv3x3"], "lic_3x3_all": ["lic_conv3x3", "lic_latent", "lic_stack"]}

    def stat(keys):
        n = sum(fam[k][0] for k in keys if k in fam)
        t = sum(fam[k][1] for k in keys if k in fam)
        fl = sum(fam[k][2] for k in keys if k in fam)
        ach = fl / t if t > 0 else 0.0
        return {"launches": n, "time_us": round(t * 1e6, 1), "gflop": round(fl / 1e9, 3),
                "achieved": round(ach / 1e12, 2), "frac": round(ach / PEAK_BF16, 4)}

    per = {k: stat([k]) for k in sorted(fam)}
    total_t = sum(v[1] for v in fam.values())  # replayed families only (entropy models / ids excluded)
    dom = max(fam, key=lambda k: fam[k][1] if fam[k][2] > 0 else -1)
    d = stat([dom])
    desc = {"lic_conv3x3": " (conv_halo_kernel + conv-source GEMM tiles: h_a / h_s)",
            "lic_latent": " (lic_latent_kernel: the slice stacks' latent-channel partial sums)",
            "lic_stack": " (lic_stack_kernel: whole cc_transform_mean/scale stacks, each serial slice's mean "
                         "stack chained into its lrp_transform stack, one workgroup per problem x image)"}
    flops_launch = d["gflop"] * 1e9 / max(d["launches"], 1)
    roof = {"kernel": dom + desc.get(dom, ""),
            "bound": "mfma", "achieved": d["achieved"], "peak": PEAK_BF16 / 1e12, "unit": "TFLOP/s",
            "frac": d["frac"], "traffic": None, "launches_per_step": d["launches"],
            "avg_launch_us": round(d["time_us"] / max(d["launches"], 1), 2),
            "flops_per_launch": round(flops_launch),
            "share_of_kernel_time": round(fam[dom][1] / total_t, 4),
            "kernel_time_per_step_us": round(total_t * 1e6, 1)}
    if dom in getattr(lt, "live_us", {}):
        # headline = the kernel as it runs INSIDE the forward (HIP events around each of its launches on its stream,
        # beside the side stream's partial sums); the back-to-back replay of the family alone stays as a second figure
        us = lt.live_us[dom]
        roof.update({"achieved": round(flops_launch / (us * 1e-6) / 1e12, 2),
                     "frac": round(flops_launch / (us * 1e-6) / PEAK_BF16, 4), "avg_launch_us": round(us, 2),
                     "measured": "in the forward: HIP events around each launch on its stream (eager forward, the "
                                 "partial sums running beside it on the side stream)",
                     "achieved_replay": d["achieved"], "frac_replay": d["frac"],
                     "avg_launch_us_replay": round(d["time_us"] / max(d["launches"], 1), 2)})
    for side in ("enc", "dec"):
        # qkv GEMM + attention core + proj; the bf16 forward runs qkv + core as ONE fused launch ({side}_qkv_attn)
        roof[f"attention_block_{side}"] = stat([f"{side}_qkv", f"{side}_attn_core", f"{side}_qkv_attn", f"{side}_proj"])
        if f"{side}_attn_core" in fam:
            roof[f"attention_core_{side}"] = stat([f"{side}_attn_core"])
        if f"{side}_qkv_attn" in fam:
            roof[f"qkv_attn_fused_{side}"] = stat([f"{side}_qkv_attn"])
    roof["families"] = per
    roof["aggregates"] = {k: stat(v) for k, v in agg.items()}
    if dom in ("lic_conv3x3", "lic_stack"):
        roof["algorithmic_bytes_per_launch"] = int((lt.conv_bytes if dom == "lic_conv3x3" else lt.stack_bytes)
                                                   / max(d["launches"], 1))
    # HBM counters (two rocprofv3 PMC passes, tools/pmc_family.py) and the graph-replayed forward's kernel trace
    # (tools/family_summary.py --forward), both committed under profiles/ from a run of this code
    # (committed for the default workload only: another model / batch gets no counter or trace figures)
    pmc, pmc_src = _committed("pmc_families.json") if profiled else (None, None)
    trace, trace_src = _committed("trace_families.json") if profiled else (None, None)
    if not profiled:
        roof["sources"] = None
        roof["sources_note"] = "profiles/ hold PMC / trace families of the default workload only (config 2, batch 64)"
    fam_pmc = (pmc or {}).get("per_family", {})
    if dom in fam_pmc:
        roof["traffic"] = fam_pmc[dom]["hbm_bytes_per_launch"]
        roof["traffic_source"] = pmc_src
    fwd = (trace or {}).get("forward", {}).get("families", {})
    rep = (trace or {}).get("replay", {}).get("families", {})
    if dom in fwd:
        us = fwd[dom]["avg_launch_us"]
        roof["frac_in_forward"] = round(roof["flops_per_launch"] / (us * 1e-6) / PEAK_BF16, 4)
        roof["avg_launch_us_in_forward"] = us
        roof["trace_source"] = trace_src
    if dom in rep:
        roof["avg_launch_us_replay_trace"] = rep[dom]["avg_launch_us"]
    # memory-bound families against the HBM roofline: algorithmic bytes / replayed kernel time
    hbm = {}
    for f, nbytes in sorted(lt.hbm_bytes.items()):
        if f not in fam:
            continue
        n, t = fam[f][0], fam[f][1]
        gbs = nbytes / t / 1e9 if t > 0 else 0.0
        e = {"launches": n, "time_us": round(t * 1e6, 1), "algorithmic_bytes_per_launch": int(nbytes / max(n, 1)),
             "achieved": round(gbs, 1), "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": round(gbs * 1e9 / PEAK_HBM, 4)}
        if f in fam_pmc:
            # normalised per forward: a PMC family can hold more kernels per ABI call than the launch timer counts
            # (eb_likelihood = eb_prep_kernel + eb_likelihood_kernel per tmae_eb_likelihood_fwd call)
            fp = fam_pmc[f]
            per_fwd = fp.get("hbm_bytes_per_fwd", fp["hbm_bytes_per_launch"] * fp.get("launches_per_fwd", n))
            e["traffic"] = int(per_fwd / max(n, 1))
            e["traffic_bytes_per_fwd"] = int(per_fwd)
            e["kernels_per_fwd_pmc"] = fp.get("launches_per_fwd")
            e["traffic_over_algorithmic"] = round(per_fwd / max(nbytes, 1), 3)
        if f in fwd:
            e["avg_launch_us_in_forward"] = fwd[f]["avg_launch_us"]
            e["frac_in_forward"] = round(nbytes / max(n, 1) / (fwd[f]["avg_launch_us"] * 1e-6) / PEAK_HBM, 4)
        hbm[f] = e
    roof["hbm_bound"] = hbm
    # the dense-source GEMMs (token GEMMs, patch / decoder embed, decoder pred, the 1x1 LIC GEMMs: PMC family
    # "token_gemm") -- counter bytes against their algorithmic A + W + output bytes, per forward
    if "token_gemm" in fam_pmc:
        tg = fam_pmc["token_gemm"]
        pf = tg.get("hbm_bytes_per_fwd", tg["hbm_bytes_per_launch"] * tg.get("launches_per_fwd", 1))
        roof["token_gemm_traffic"] = {
            "launches_per_fwd_classified": lt.gemm_bytes[0], "launches_per_fwd_pmc": tg.get("launches_per_fwd"),
            "algorithmic_bytes_per_fwd": int(lt.gemm_bytes[1]), "traffic_bytes_per_fwd": int(pf),
            "traffic_over_algorithmic": round(pf / max(lt.gemm_bytes[1], 1), 3), "source": pmc_src}
    if pmc_src or trace_src:
        roof["sources"] = {"pmc": pmc_src, "trace": trace_src}
    return roof


def _committed(name):
    """the newest profiles/rNN/<name> (committed evidence), parsed, and its repo-relative path"""
    base = os.path.join(ROOT, "profiles")
    try:
        rounds = sorted(d for d in os.listdir(base) if d.startswith("r") and d[1:].isdigit())
    except OSError:
        return None, None
    for d in reversed(rounds):
        p = os.path.join(base, d, name)
        if os.path.exists(p):
            try:
                return json.load(open(p)), os.path.relpath(p, ROOT)
            except Exception:
                return None, None
    return None, None


def train_bench(model, args, rank, world, dev, barrier):
    """the reference training step (utils/engine.py:72-91): forward, RateDistortionLoss (SSIM + L1 +
    bpp; VGG needs a weight download), aux loss, backward (HIP reverse pass; for world > 1 the RCCL
    gradient all-reduce runs inside it, bucketed), clip_grad_norm_(1.0), Adam, aux backward, aux Adam.
    The whole step is one HIP graph (engine.GraphedTrainStep), replayed per batch, at any world size over RCCL:
    the bucketed gradient all-reduces are captured inside the backward; the crop kernel runs before each
    replay.  The all-reduce overlap numbers (parallel.GradSync.last_timing) come from one eager step of the same
    kernels after the timed replays.  A gloo group (CPU rehearsals) runs eager steps."""
    from textmae_amd import engine
    from textmae_amd.data import SyntheticCropSet
    from textmae_amd.optim import configure_optimizers
    from textmae_amd.parallel import enable_data_parallel
    from textmae_amd.rd_loss import RateDistortionLoss

    model.train()
    model.distortion = "ssim+l1"
    if world > 1:
        enable_data_parallel(model, timing=True)
    opt, aux_opt = configure_optimizers(model, lr=1e-4, aux_lr=1e-4, fused=True)
    crit = RateDistortionLoss(lmbda=1e-2)
    # BASELINE config 3's input: per rank, seeded DIV2K-shaped uint8 images (2040 x 1356) resident in HBM and
    # a fresh random 256^2 crop per sample per step, ToTensor + Normalize on the device (data.py); seed =
    # base + rank as training.py:109 seeds its processes
    data = SyntheticCropSet(dev, seed=2000, rank=rank, crop=args.img,
                            patch_size=model.encoder_embed.patch_size[0]).plan(args.train_warmup + args.train_steps + 1,
                                                                               args.train_batch)
    use_graph = not args.no_graph and (world == 1 or args.backend == "nccl")
    if use_graph:
        imgs, scores = data.next()
        gstep = engine.GraphedTrainStep(model, crit, opt, aux_opt, imgs, scores, clip_max_norm=1.0, warmup=1)

        def step():
            imgs, scores = data.next()
            return gstep(imgs, scores)
    else:
        def step():
            imgs, scores = data.next()
            return engine.train_step(model, crit, imgs, scores, opt, aux_opt, clip_max_norm=1.0)

    for _ in range(args.train_warmup):
        out = step()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        out = step()
    host = time.perf_counter() - t0  # the host's enqueue time: close to the wall time = launch-bound
    torch.cuda.synchronize()
    barrier()
    el = max_over_ranks(time.perf_counter() - t0, world, dev, args.backend)
    ips = world * args.train_batch * args.train_steps / el
    fl = 3 * sum(gflop_per_image(model).values())
    rec = {"metric": "training images/s (fwd + bwd + clip + 2x Adam" + (", RCCL grad all-reduce" if world > 1 else "")
           + ")", "value": round(ips, 2), "unit": "images/s", "ms_per_step": round(el / args.train_steps * 1e3, 3),
           "host_enqueue_ms_per_step": round(host / args.train_steps * 1e3, 3),
           "steps": args.train_steps, "warmup": args.train_warmup, "per_gpu_batch": args.train_batch,
           "global_batch": args.train_batch * world, "parallelism": f"dp{world}", "dtype": "bf16",
           "data": f"DIV2K-shaped: {data.images.shape[0]} seeded uint8 2040x1356 images per rank (seed 2000 + rank), "
                   f"a random {args.img}^2 crop per sample per step, normalised on the device",
           "loss_last": round(float(out["loss"].detach()), 6), "gflop_per_image": round(fl, 2),
           "step_mfma_frac": round(ips * fl * 1e9 / (world * PEAK_BF16), 4), "hip_graph": use_graph}
    if use_graph:
        del gstep
        torch.cuda.empty_cache()
    if world > 1:
        if use_graph:  # the captured step records no events: one eager step of the same kernels for the overlap
            imgs, scores = data.next()
            engine.train_step(model, crit, imgs, scores, opt, aux_opt, clip_max_norm=1.0)
        t = model.grad_sync.last_timing()
        if t:
            rec["grad_allreduce"] = dict(t, source="this rank's compute-stream events, " + (
                "one eager step after the timed graph replays" if use_graph else "last timed step"))
    elif args.dp_rehearsal:
        rec["grad_allreduce"] = dp_rehearsal(model, crit, opt, aux_opt, data, dev)
    return rec


def dp_rehearsal(model, crit, opt, aux_opt, data, dev, steps=3):
    """the data-parallel step's overlap numbers at N = 1: an RCCL process group of ONE rank
    with GradSync's world-of-1 short-circuit bypassed, so the bucketed async AVG all-reduces really go through
    RCCL from inside the backward; a few eager steps, then the last one's events.  A one-rank all-reduce moves
    no bytes over xGMI: this measures the issue / overlap structure, not link time."""
    import torch.distributed as dist

    from textmae_amd import engine
    from textmae_amd.parallel import enable_data_parallel

    own = not dist.is_initialized()
    try:
        if own:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=dev)
        sync = enable_data_parallel(model, always_collective=True, timing=True)
        for _ in range(steps):
            imgs, scores = data.next()
            engine.train_step(model, crit, imgs, scores, opt, aux_opt, clip_max_norm=1.0)
        torch.cuda.synchronize()
        t = sync.last_timing()
        rec = dict(t or {}, launched_total=sync.launched, world=1,
                   source="one-rank nccl (RCCL) group, always_collective, last of 3 eager steps")
        # the DP step as the N > 1 ranks run it: ONE HIP graph holding the bucketed RCCL all-reduces
        n0 = sync.launched
        imgs, scores = data.next()
        gstep = engine.GraphedTrainStep(model, crit, opt, aux_opt, imgs, scores, clip_max_norm=1.0, warmup=1)
        captured = sync.launched - n0
        for _ in range(2):
            gstep(*data.next())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            gstep(*data.next())
        host = time.perf_counter() - t0
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rec["graphed"] = {"hip_graph": True, "ms_per_step": round(el / steps * 1e3, 3),
                          "host_enqueue_ms_per_step": round(host / steps * 1e3, 3),
                          "collectives_in_graph": captured - (len(sync._bounds) - 1),  # minus the warm-up step's
                          "buckets_issued_in_backward": sync.launched_in_backward,
                          "source": f"GraphedTrainStep with the one-rank RCCL GradSync, {steps} replays"}
        del gstep
        return rec
    except Exception as e:  # the rehearsal must never cost the bench line
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    finally:
        model.grad_sync = None
        if own and dist.is_initialized():
            dist.destroy_process_group()


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cpu_leg(threads, seconds, max_batches, batch, model_kwargs):
    """one timed leg of the CPU baseline (runs in a child process: see cpu_baseline)"""
    from oracle.mcm_oracle import MCMConfig, make_state_dict, mcm_forward

    torch.set_num_threads(threads)
    cfg = MCMConfig(**model_kwargs)
    sd = make_state_dict(cfg, 0)
    L = (cfg.img_size // cfg.patch_size) ** 2
    x, s = synthetic_inputs(batch, cfg.img_size, L, 0, "cpu")
    mcm_forward(sd, cfg, x[:1], s[:1])  # untimed warm-up (one image): first-call allocation / primitive setup
    ts, t0 = [], time.perf_counter()
    while len(ts) < max_batches:
        t1 = time.perf_counter()
        mcm_forward(sd, cfg, x, s)
        ts.append(time.perf_counter() - t1)
        if time.perf_counter() - t0 >= seconds:
            break
    ts.sort()
    med = ts[len(ts) // 2] if len(ts) % 2 else 0.5 * (ts[len(ts) // 2 - 1] + ts[len(ts) // 2])
    return {"threads": torch.get_num_threads(), "images_per_s_median": round(batch / med, 3), "batches": len(ts),
            "batch": batch, "images_per_s_mean": round(batch * len(ts) / sum(ts), 3)}


def _cpu_share():
    """CPUs the cgroup lets this process use (cpu.max quota / period), or None"""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        return None


def cpu_baseline(args, model_kwargs):
    """the oracle (CPU restatement of MCM.forward, fp32) on the host cores over a bounded
    sample of the same workload (batches of 8), timed per batch and reported at the median:
      * at the thread count of the cgroup's CPU share (cpu.max; os.cpu_count() when there is no quota:
        §8(d)'s setting -- on the box os.cpu_count() is 256 against a 16-CPU share, and 256 threads never
        finish a batch);
      * at the thread count the process is given (OMP_NUM_THREADS; the box's CPU share);
      * at 1 thread, the reference eval convention (testing.py:29).
    Each leg runs in its own child process (no GPU use there) under a time limit, so a leg that
    oversubscribes the box's CPU share cannot stall the run; ``value`` / ``cores`` are the faster of the first
    two.  Plus the reference-semantics get_ids_shuffle alone (the C restatement of MCM.py:364-423, batch 64)."""
    import subprocess

    import numpy as np

    from oracle import ids as ids_oracle

    nb = args.cpu_batch
    default_threads = torch.get_num_threads()
    legs = {}
    # the box gives this process a cgroup CPU share (cpu.max) far below os.cpu_count(): a leg with one thread per
    # host CPU oversubscribes the share ~16x and never finishes a batch, so it is sized to the share instead
    host = os.cpu_count() or default_threads
    share = _cpu_share()
    share_threads = max(1, min(host, int(share + 0.5))) if share else host
    plan = [("cgroup_share", share_threads, args.cpu_seconds, 1000)]
    if default_threads != share_threads:
        plan.append(("process_threads", default_threads, args.cpu_seconds, 1000))
    plan.append(("one_thread", 1, 0.0, 1))
    if share_threads < host:
        legs["all_host_cpus"] = {"threads": host, "skipped": f"cgroup cpu.max share is {share} CPUs; "
                                                             f"{host} threads would oversubscribe it"}
    for name, threads, secs, maxb in plan:
        env = dict(os.environ, OMP_NUM_THREADS=str(threads))
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-leg", json.dumps([threads, secs, maxb, nb, model_kwargs])]
        limit = 4 * secs + 120
        progress(f"cpu baseline leg {name}: {threads} threads (limit {limit:.0f} s)")
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=limit, env=env)
            line = [l for l in r.stdout.splitlines() if l.startswith("{")]
            legs[name] = json.loads(line[-1]) if r.returncode == 0 and line else {"threads": threads,
                                                                                   "error": r.stderr[-300:]}
        except subprocess.TimeoutExpired:
            legs[name] = {"threads": threads, "error": f"no batch of {nb} finished within {limit:.0f} s"}
    ok = [k for k in ("cgroup_share", "process_threads") if "images_per_s_median" in legs.get(k, {})]
    best = max(ok, key=lambda k: legs[k]["images_per_s_median"]) if ok else None
    L = (model_kwargs["img_size"] // 16) ** 2
    s64 = torch.rand(64, L, generator=torch.Generator().manual_seed(5)).numpy().astype(np.float32)
    ids_oracle.ids_shuffle(s64, model_kwargs["num_keep_patches"])
    reps, t2 = 0, time.perf_counter()
    while time.perf_counter() - t2 < 1.0:
        ids_oracle.ids_shuffle(s64, model_kwargs["num_keep_patches"])
        reps += 1
    ids_ms = (time.perf_counter() - t2) / reps * 1e3
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:
        aff = None
    return {"value": legs[best]["images_per_s_median"] if best else None, "unit": "images/s",
            "cores": legs[best]["threads"] if best else None, "kind": "port",
            "sample": f"oracle MCM.forward (fp32 torch CPU restatement) on batches of {nb} at "
                      f"{model_kwargs['img_size']}^2, K={model_kwargs['num_keep_patches']}, timed per batch, median; "
                      f"~{args.cpu_seconds:.0f} s per multi-thread leg, one batch at 1 thread; value = the faster of "
                      f"the cgroup CPU share's threads and the process's threads",
            "legs": legs, "value_1thread": legs["one_thread"].get("images_per_s_median"), "cpu_model": _cpu_model(),
            "host_cpus": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_share": _cpu_share(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "ids_shuffle_ms_per_batch64_1thread": round(ids_ms, 3)}


def progress(msg):
    """phase markers on stderr (a long bench keeps its output flowing; stdout carries only the JSON line)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def time_forward(model, imgs, scores, steps, warmup, use_graph, world, dev, backend, barrier):
    """the timed region: `warmup` untimed forwards, then exactly `steps` forwards (replays of one HIP graph)
    between barrier + synchronize on both sides; returns (max-over-ranks wall seconds, median step ms from
    per-step HIP events recorded on the stream -- no host sync inside the region)"""
    graph = None
    with torch.no_grad():
        if use_graph:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    model(imgs, scores)
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                model(imgs, scores)

            def step():
                graph.replay()
        else:
            def step():
                model(imgs, scores)

        for _ in range(warmup):
            step()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record()
        for i in range(steps):
            step()
            evs[i + 1].record()
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.perf_counter() - t0, world, dev, backend)
    ms = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    med = ms[len(ms) // 2] if len(ms) % 2 else 0.5 * (ms[len(ms) // 2 - 1] + ms[len(ms) // 2])
    del graph
    return el, med


def k64_line(args, dev, world, rank, barrier, dtype):
    """SURVEY §8(d) config 2's secondary point: the same ViT-B model at K=64 kept patches (mask 0.75, g=8),
    batch 64, timed exactly like the main line"""
    import textmae_amd

    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=args.img, num_keep_patches=64).to(dev).eval()
    m.compute_dtype = dtype
    m.distortion = "none"
    L = m.encoder_embed.num_patches
    imgs, scores = synthetic_inputs(args.batch, args.img, L, 1000 + rank, dev)
    el, med = time_forward(m, imgs, scores, args.steps, args.warmup, not args.no_graph, world, dev, args.backend,
                           barrier)
    gf = sum(gflop_per_image(m).values())
    v = world * args.batch * args.steps / el
    del m
    torch.cuda.empty_cache()
    return {"workload": "MCM forward eval, ViT-B/16, K=64 of 256 patches (g=8)", "value": round(v, 2),
            "unit": "images/s", "ms_per_step": round(el / args.steps * 1e3, 3), "ms_per_step_median": round(med, 3),
            "gflop_per_image": round(gf, 3), "step_mfma_frac": round(v * gf * 1e9 / (world * PEAK_BF16), 4)}


def seeded_vgg16_features(seed=0):
    """VGG16 features[0:16] conv weights of torchvision's layout, seeded (kaiming-normal, zero bias): the
    pretrained ones need a download (loss/vgg.py:14), so the timing line runs the same architecture on
    random-init weights, as every other line here does"""
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for i, (ci, co) in zip((0, 2, 5, 7, 10, 12, 14), ((3, 64), (64, 64), (64, 128), (128, 128), (128, 256),
                                                    (256, 256), (256, 256))):
        sd[f"features.{i}.weight"] = torch.randn(co, ci, 3, 3, generator=g) * (2.0 / (9 * ci)) ** 0.5
        sd[f"features.{i}.bias"] = torch.zeros(co)
    return sd


def distortion_line(model, imgs, scores, args, world, dev, barrier):
    """MCM.forward_loss (MCM.py:690-712: 1 - SSIM, L1, VGG16 relu2_2 / relu3_3 feature loss)
    timed on its own, apart from the encode + rate + decode metric: one forward gives x_hat, then exactly
    `steps` replays of a HIP graph of forward_loss(imgs, x_hat) at the bench batch (eval, no_grad)"""
    model.load_vgg16(seeded_vgg16_features(0))
    with torch.no_grad():
        x_hat = model(imgs, scores)["x_hat"].clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                model.forward_loss(imgs, x_hat)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = model.forward_loss(imgs, x_hat)
        for _ in range(args.warmup):
            graph.replay()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            graph.replay()
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.perf_counter() - t0, world, dev, args.backend)
        vals = [round(float(v), 6) for v in out]
    del graph
    model.__dict__["_vgg_sd"] = None
    model.__dict__["_vgg"] = None
    B, H = imgs.shape[0], imgs.shape[-1]
    # VGG16 features[0:16] FLOPs for prediction and target (2 MAC per tap)
    vgg = 0
    hw = H * H
    for ci, co, pool_before in ((3, 64, 0), (64, 64, 0), (64, 128, 1), (128, 128, 0), (128, 256, 1), (256, 256, 0),
                                (256, 256, 0)):
        hw //= 4 if pool_before else 1
        vgg += 2 * hw * co * ci * 9
    gf = 2 * vgg / 1e9
    v = world * B * args.steps / el
    return {"workload": "MCM.forward_loss: 1 - SSIM (11x11 Gaussian, 3 channels) + L1 + VGG16 features[0:16] "
                        "feature MSE on prediction and target (seeded VGG weights), eval, HIP graph",
            "value": round(v, 2), "unit": "images/s", "ms_per_step": round(el / args.steps * 1e3, 3),
            "batch": B, "gflop_per_image": round(gf, 3), "step_mfma_frac": round(v * gf * 1e9 / (world * PEAK_BF16), 4),
            "losses": {"ssim_loss": vals[0], "L1_loss": vals[1], "vgg_loss": vals[2]}}


def mae_large_line(args, dev, world, rank, barrier, dtype):
    """BASELINE config 4 as written: MAE ViT-Large (mae_vit_large_patch16_dec512d8b, models_mae.py:231-236:
    1024/24/16 encoder, decoder 512/8/16), batch 128, 224^2, mask_ratio 0.75, forward (masking, encoder on the 49
    kept patches, decoder, masked MSE loss) replayed as a HIP graph; seeded random-init weights"""
    import textmae_amd

    torch.manual_seed(0)
    m = textmae_amd.mae_vit_large_patch16_dec512d8b().to(dev).eval()
    m.compute_dtype = dtype
    B = 128
    imgs = torch.randn(B, 3, 224, 224, generator=torch.Generator().manual_seed(2000 + rank)).to(dev)
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                m(imgs, 0.75)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            m(imgs, 0.75)
        for _ in range(args.warmup):
            graph.replay()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            graph.replay()
        torch.cuda.synchronize()
        barrier()
        el = max_over_ranks(time.perf_counter() - t0, world, dev, args.backend)
    del graph
    L, keep, E, Dd = 196, 49, 1024, 512
    fl = 2 * keep * E * 768  # patch embed of the kept patches
    fl += 24 * (2 * (keep + 1) * E * 12 * E + 4 * (keep + 1) ** 2 * E)
    fl += 2 * (keep + 1) * E * Dd
    fl += 8 * (2 * (L + 1) * Dd * 12 * Dd + 4 * (L + 1) ** 2 * Dd)
    fl += 2 * L * Dd * 768
    gf = fl / 1e9
    v = world * B * args.steps / el
    del m
    torch.cuda.empty_cache()
    return {"workload": "BASELINE config 4: MAE ViT-Large/16 dec512d8b forward (mask 0.75, loss), 224^2, HIP graph",
            "value": round(v, 2), "unit": "images/s", "batch": B, "ms_per_step": round(el / args.steps * 1e3, 3),
            "dtype": "bf16" if dtype == torch.bfloat16 else "f32", "gflop_per_image": round(gf, 3),
            "step_mfma_frac": round(v * gf * 1e9 / (world * PEAK_BF16), 4)}


def mae_train_line(args, dev, world, rank, barrier, dtype):
    """MaskedAutoencoderViT training step (models_mae.py:216-220 under autograd; mae_train.py): forward with the
    activations kept, masked-MSE loss, HIP backward of the whole model, FusedAdam; mae_vit_base_patch16_dec512d8b,
    batch 64, 224^2, mask_ratio 0.75, the step replayed as one HIP graph (engine.GraphedMAEStep); seeded
    random-init weights and images"""
    import textmae_amd
    from textmae_amd import engine
    from textmae_amd.optim import FusedAdam

    torch.manual_seed(0)
    m = textmae_amd.mae_vit_base_patch16_dec512d8b().to(dev).train()
    m.compute_dtype = dtype
    B, steps = 64, 10
    imgs = torch.randn(B, 3, 224, 224, generator=torch.Generator().manual_seed(3000 + rank)).to(dev)
    opt = FusedAdam([p for p in m.parameters() if p.requires_grad], lr=1.5e-4)
    step = engine.GraphedMAEStep(m, opt, imgs, 0.75, warmup=2)  # fresh masking noise per replay
    step(imgs)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step(imgs)
    torch.cuda.synchronize()
    barrier()
    el = max_over_ranks(time.perf_counter() - t0, world, dev, args.backend)
    L, keep, E, Dd = 196, 49, 768, 512
    fl = 2 * keep * E * 768
    fl += 12 * (2 * (keep + 1) * E * 12 * E + 4 * (keep + 1) ** 2 * E)
    fl += 2 * (keep + 1) * E * Dd
    fl += 8 * (2 * (L + 1) * Dd * 12 * Dd + 4 * (L + 1) ** 2 * Dd)
    fl += 2 * L * Dd * 768
    gf = 3 * fl / 1e9  # forward + the two backward GEMM passes
    v = world * B * steps / el
    out = {"workload": "MAE ViT-Base/16 dec512d8b training step (forward + masked MSE + HIP backward + FusedAdam), "
                       "224^2, mask 0.75, HIP graph", "value": round(v, 2), "unit": "images/s", "batch": B,
           "ms_per_step": round(el / steps * 1e3, 3), "dtype": "bf16" if dtype == torch.bfloat16 else "f32",
           "gflop_per_image": round(gf, 3), "step_mfma_frac": round(v * gf * 1e9 / (world * PEAK_BF16), 4),
           "loss_last": round(float(loss), 6), "hip_graph": True}
    del step, m, opt
    torch.cuda.empty_cache()
    return out


def max_over_ranks(el, world, dev, backend):
    if world <= 1:
        return el
    t = torch.tensor([el], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def _free_port():
    import socket

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(args):
    """``--gpus N`` (N > 1) without a torch.distributed launcher: start the N ranks here, one process per
    GPU, through torch.distributed.run on 127.0.0.1, and return its exit code.  The parent never touches
    the GPU (torch.cuda.device_count() does not initialise it), so nothing is exec'ed after a GPU call."""
    import subprocess

    if args.backend == "nccl" and torch.cuda.device_count() < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but only {torch.cuda.device_count()} GPU(s) visible", file=sys.stderr)
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def main():
    args = parse()
    if args.cpu_leg:
        threads, secs, maxb, nb, kw = json.loads(args.cpu_leg)
        print(json.dumps(_cpu_leg(threads, secs, maxb, nb, kw)), flush=True)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    local = int(os.environ.get("LOCAL_RANK", 0))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    import textmae_amd

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    torch.manual_seed(0)
    kw = dict(img_size=args.img, num_keep_patches=args.keep, encoder_embed_dim=args.enc_dim,
              encoder_depth=args.enc_depth, encoder_num_heads=args.enc_heads)
    model = textmae_amd.MCM(**kw).to(dev).eval()
    model.compute_dtype = dtype
    model.distortion = "none"  # metric = encode + rate + decode; forward_loss is reported separately
    L = model.encoder_embed.num_patches
    imgs, scores = synthetic_inputs(args.batch, args.img, L, 1000 + rank, dev)
    gf = gflop_per_image(model)
    gf_img = sum(gf.values())

    progress(f"forward: batch {args.batch}, {args.steps} timed steps")
    el, med_ms = time_forward(model, imgs, scores, args.steps, args.warmup, not args.no_graph, world, dev, args.backend,
                              barrier)
    roof = None
    if rank == 0 and not args.no_roofline:
        progress("roofline: per-family replays")
        roof = roofline_report(model, imgs, scores, args.batch, dump=args.dump_launches,
                               profiled=vitb_default(args) and args.batch == 64 and args.img == 256)

    k64 = None
    if args.k64_line and vitb_default(args):
        progress("config 2' (K=64) line")
        k64 = k64_line(args, dev, world, rank, barrier, dtype)

    mae_l = None
    if args.mae_large:
        progress("config 4 (MAE ViT-L, batch 128) line")
        mae_l = mae_large_line(args, dev, world, rank, barrier, dtype)

    mae_t = None
    if args.mae_train_line and vitb_default(args) and world == 1:
        progress("MAE ViT-B training line")
        mae_t = mae_train_line(args, dev, world, rank, barrier, dtype)

    dist_line = None
    if args.distortion_line and vitb_default(args):
        progress("forward_loss line")
        dist_line = distortion_line(model, imgs, scores, args, world, dev, barrier)

    train = None
    if not args.no_train and args.train_steps > 0:
        progress("training step")
        train = train_bench(model, args, rank, world, dev, barrier)

    vitb = args.enc_dim == 768 and args.enc_depth == 12
    value = world * args.batch * args.steps / el
    rec = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 3),
        "ms_per_step_median": round(med_ms, 3), "value_at_median": round(world * args.batch / (med_ms * 1e-3), 2),
        "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded uniform RGB, "
        "ImageNet-normalised; uniform patch scores; seeded random-init weights)",
        "config": {"workload": ("MCM forward eval: ids+ViT-B/16 enc" if vitb else
                                f"BASELINE config 4 MCM forward eval: ids+ViT enc {args.enc_dim}/{args.enc_depth}/"
                                f"{args.enc_heads}") + f" (K={args.keep} of {L} patches) + LIC hyperprior + EB/GC "
                                "rates + ViT dec 512/8/16 + unpatchify",
                   "img_size": args.img, "num_keep_patches": args.keep, "per_gpu_batch": args.batch,
                   "global_batch": args.batch * world, "parallelism": f"replicas x{world}",
                   "hip_graph": not args.no_graph},
        "gflop_per_image": round(gf_img, 3),
        "step_mfma_frac": round(value * gf_img * 1e9 / (world * PEAK_BF16), 4),
        "roofline": roof,
    }
    if k64 is not None:
        rec["config2_k64"] = k64
    if dist_line is not None:
        rec["forward_loss"] = dist_line
    if mae_l is not None:
        rec["config4_mae_large"] = mae_l
    if mae_t is not None:
        rec["mae_train"] = mae_t
    if train is not None:
        rec["train"] = train
    if rank == 0:
        if world == 1 and not args.no_cpu_baseline:
            progress("cpu baseline")
            rec["cpu_baseline"] = cpu_baseline(args, kw)
        print(json.dumps(rec), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
