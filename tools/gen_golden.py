"""Generate golden fixtures from the REAL reference code (run only in the survey container, where
/root/reference exists; the fixtures it writes under tests/golden/ are small data files).

The reference's own Python is imported by path.  Its third-party imports (compressai, timm,
pytorch_msssim, torchvision — none installed) are satisfied with the oracle's
restatements from oracle/thirdparty.py, so what these fixtures pin is the reference GLUE:
get_ids_shuffle (bit-exact ids), random_masking, the LIC slice loop and tensor layouts, the decoder
unshuffle with its off-by-one cls, unpatchify, RateDistortionLoss and the sin-cos tables.

    python tools/gen_golden.py            # writes tests/golden/*.npz
"""
from __future__ import annotations

import hashlib
import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("TMAE_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)

from oracle import thirdparty as tp  # noqa: E402
from oracle.mcm_oracle import MCMConfig, make_state_dict  # noqa: E402


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class _NoCoder:  # compressai.ans is C++ upstream; not needed for forward()
        def __init__(self, *a, **k):
            raise RuntimeError("rANS coder not available in the golden generator")

    mod("compressai")
    mod("compressai.ans", BufferedRansEncoder=_NoCoder, RansDecoder=_NoCoder)
    mod("compressai.entropy_models", EntropyBottleneck=tp.EntropyBottleneck, GaussianConditional=tp.GaussianConditional)
    mod("compressai.layers", conv3x3=tp.conv3x3, subpel_conv3x3=tp.subpel_conv3x3)
    mod("compressai.models", CompressionModel=tp.CompressionModel)
    mod("compressai.ops", quantize_ste=tp.quantize_ste)
    mod("pytorch_msssim", SSIM=tp.SSIM, ms_ssim=None)
    mod("timm")
    mod("timm.models")
    mod("timm.models.vision_transformer", PatchEmbed=tp.PatchEmbed, Block=tp.Block)
    # VGG16 needs torchvision + a pretrained download: the feature loss is replaced by 0 here.
    mod("models.Compression.loss.vgg", cal_features_loss=lambda a, b: torch.zeros((), dtype=a.dtype))
    if not hasattr(np, "float_"):
        np.float_ = np.float64  # pos_embed.py:83 uses the numpy<2 alias
    sys.path.insert(0, REF)


def sha16(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


# ---------------------------------------------------------------------------------------- F1
def score_cases(rng, L, kind, count):
    out = []
    for _ in range(count):
        if kind == "uniform":
            s = rng.random(L, dtype=np.float32)
        elif kind == "ties":
            # generate_scores_file.py:19-29: product of two patch-mean maps, min-max normalised
            t = rng.integers(0, 40, L).astype(np.float32)
            u = rng.integers(1, 12, L).astype(np.float32)
            s = t * u
            s = (s - s.min()) / (s.max() - s.min())
        elif kind == "fewuniq":  # few unique values -> empty groups -> NaN means
            s = rng.choice(np.array([0.0, 0.25, 0.5, 1.0], dtype=np.float32)[: rng.integers(2, 5)], L)
        elif kind == "skewed":  # heavy top decile: K - |group9| small or negative; slice wrap
            s = rng.random(L, dtype=np.float32) ** 8
            s[rng.random(L) < 0.4] = 1.0
        elif kind == "zeros":  # mostly zeros with a few values (signed zero too)
            s = np.zeros(L, dtype=np.float32)
            idx = rng.choice(L, size=rng.integers(1, L // 4), replace=False)
            s[idx] = rng.random(len(idx), dtype=np.float32)
            s[rng.choice(L, 3, replace=False)] = -0.0
        out.append(s.astype(np.float32))
    return np.stack(out)


def gen_ids(MCM):
    rng = np.random.default_rng(1234)
    data = {}
    combos = [(196, 144), (196, 64), (196, 49), (256, 144), (256, 64), (256, 49), (64, 16), (16, 4), (256, 256)]
    kinds = ["uniform", "ties", "fewuniq", "skewed", "zeros"]
    for L, K in combos:
        for kind in kinds:
            n = 24 if L >= 196 else 12
            s = score_cases(rng, L, kind, n)
            ids = MCM.get_ids_shuffle(SimpleNamespace(num_keep_patches=K), torch.from_numpy(s)).numpy()
            assert ids.shape == (n, L) and all(sorted(r) == list(range(L)) for r in ids.tolist())
            key = f"L{L}_K{K}_{kind}"
            data[key + "_scores"] = s
            data[key + "_ids"] = ids.astype(np.int16)
    np.savez_compressed(os.path.join(OUT, "ids_shuffle.npz"), **data)
    print("ids_shuffle.npz:", len(combos) * len(kinds), "groups")


# ---------------------------------------------------------------------------------------- F3
def gen_pos():
    from models.Compression.common.pos_embed import get_2d_sincos_pos_embed

    data = {}
    for d, g in [(768, 16), (512, 16), (768, 14), (1024, 16), (64, 8), (32, 8)]:
        pe = get_2d_sincos_pos_embed(d, g, cls_token=True).astype(np.float32)
        data[f"d{d}_g{g}_sha"] = np.array(sha16(pe))
        data[f"d{d}_g{g}_rows"] = pe[[0, 1, g + 3, g * g]]
    np.savez_compressed(os.path.join(OUT, "pos_embed.npz"), **data)
    print("pos_embed.npz")


# ---------------------------------------------------------------------------------------- F4/F5
TINY = dict(img_size=128, patch_size=16, encoder_embed_dim=64, encoder_depth=2, encoder_num_heads=2,
            decoder_embed_dim=32, decoder_depth=2, decoder_num_heads=1, latent_depth=64, hyperprior_depth=32,
            num_slices=4, num_keep_patches=16)
SMALL12 = dict(img_size=128, patch_size=16, encoder_embed_dim=128, encoder_depth=1, encoder_num_heads=2,
               decoder_embed_dim=64, decoder_depth=1, decoder_num_heads=2, latent_depth=192, hyperprior_depth=96,
               num_slices=12, num_keep_patches=16)


def gen_forward(MCM, name, cfgd, batch, seed):
    from models.Compression.loss.rd_loss import RateDistortionLoss

    cfg = MCMConfig(**cfgd)
    sd = make_state_dict(cfg, seed)
    ref = MCM(**cfg.kwargs())
    full = ref.state_dict()
    missing = [k for k in full if k not in sd and not k.endswith("bound") and not k.startswith(
        ("entropy_bottleneck._", "gaussian_conditional."))]
    assert not missing, missing
    full.update(sd)
    ref.load_state_dict(full)
    rng = np.random.default_rng(seed + 1)
    L = (cfg.img_size // cfg.patch_size) ** 2
    imgs = rng.random((batch, 3, cfg.img_size, cfg.img_size), dtype=np.float32)
    scores = score_cases(rng, L, "ties", batch)
    g = int(cfg.num_keep_patches ** 0.5)
    hz = (((g + 1) // 2) + 1) // 2
    z_noise = rng.uniform(-0.5, 0.5, (batch, cfg.hyperprior_depth, hz, hz)).astype(np.float32)
    y_noise = rng.uniform(-0.5, 0.5, (batch, cfg.latent_depth, g, g)).astype(np.float32)
    data = dict(imgs=imgs, scores=scores, z_noise=z_noise, y_noise=y_noise,
                weights_sha=np.array(sha16(np.concatenate([v.numpy().ravel() for v in sd.values()]))))
    crit = RateDistortionLoss(lmbda=1e-4)
    with torch.no_grad():
        for mode in ("eval", "train"):
            if mode == "eval":
                ref.eval()
            else:
                ref.train()
                ref.entropy_bottleneck.noise_queue = [torch.from_numpy(z_noise)]
                ref.gaussian_conditional.noise_queue = list(torch.from_numpy(y_noise).chunk(cfg.num_slices, 1))
            t = torch.from_numpy(imgs)
            out = ref(t, torch.from_numpy(scores))
            _, rest = ref.random_masking(torch.zeros(batch, L, 1), torch.from_numpy(scores))
            rd = crit(out, t)
            data[f"{mode}_x_hat"] = out["x_hat"].numpy()
            data[f"{mode}_y_lik"] = out["likelihoods"]["y"].numpy()
            data[f"{mode}_z_lik"] = out["likelihoods"]["z"].numpy()
            data[f"{mode}_ids_restore"] = rest.numpy()
            data[f"{mode}_ssim_loss"] = np.float32(out["loss"][0])
            data[f"{mode}_l1_loss"] = np.float32(out["loss"][1])
            data[f"{mode}_bpp_loss"] = np.float32(rd["bpp_loss"])
            data[f"{mode}_loss"] = np.float32(rd["loss"])
        data["aux_loss"] = np.float32(ref.aux_loss())
    np.savez_compressed(os.path.join(OUT, f"mcm_{name}.npz"), **data)
    print(f"mcm_{name}.npz", {k: v.shape for k, v in data.items() if hasattr(v, 'shape')})


# ---------------------------------------------------------------------------------------- F6
def gen_mae_masking():
    mm = _ref_mae_module()
    data = {}
    for seed in (0, 1, 2):
        torch.manual_seed(seed)
        x = torch.arange(4 * 196, dtype=torch.float32).reshape(4, 196, 1)
        xm, mask, rest = mm.MaskedAutoencoderViT.random_masking(None, x, 0.75)
        data[f"s{seed}_x_masked"] = xm.numpy()
        data[f"s{seed}_mask"] = mask.numpy()
        data[f"s{seed}_ids_restore"] = rest.numpy()
    np.savez_compressed(os.path.join(OUT, "mae_masking.npz"), **data)
    print("mae_masking.npz")


def _ref_mae_module():
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_models_mae", os.path.join(REF, "models/MAE/models_mae.py"))
    mm = importlib.util.module_from_spec(spec)
    sys.modules["util.pos_embed"] = sys.modules["models.Compression.common.pos_embed"]
    spec.loader.exec_module(mm)
    return mm


def gen_mae_forward():
    """mae_vit_base_patch16_dec512d8b built after torch.manual_seed(0), imgs =
    randn(4,3,224,224) from a generator seeded 1, torch.manual_seed(2) right before forward(mask_ratio=0.75);
    plus a tiny norm_pix_loss=True model.  pred is stored on every 7th patch row (size)."""
    from functools import partial

    mm = _ref_mae_module()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    torch.manual_seed(0)
    model = mm.mae_vit_base_patch16_dec512d8b()
    sd = model.state_dict()
    init_sha = sha16(np.concatenate([v.float().numpy().ravel() for v in sd.values() if v.numel()]))
    imgs = torch.randn(4, 3, 224, 224, generator=torch.Generator().manual_seed(1))
    torch.manual_seed(2)
    noise = torch.rand(4, 196)
    torch.manual_seed(2)
    with torch.no_grad():
        loss, pred, mask = model(imgs, mask_ratio=0.75)
    data = {"init_sha_seed0": np.array(init_sha), "noise": noise.numpy(), "loss": loss.numpy(),
            "mask": mask.numpy(), "pred_rows": pred[:, ::7].numpy(), "pred_sum": pred.double().sum((1, 2)).numpy()}
    # tiny norm_pix_loss model (every shape of the path, small enough to store whole)
    torch.manual_seed(5)
    tiny = mm.MaskedAutoencoderViT(img_size=64, patch_size=16, in_chans=3, embed_dim=64, depth=2, num_heads=2,
                                   decoder_embed_dim=32, decoder_depth=1, decoder_num_heads=1, mlp_ratio=4.0,
                                   norm_layer=partial(torch.nn.LayerNorm, eps=1e-6), norm_pix_loss=True)
    timgs = torch.randn(2, 3, 64, 64, generator=torch.Generator().manual_seed(6))
    torch.manual_seed(7)
    tnoise = torch.rand(2, 16)
    torch.manual_seed(7)
    with torch.no_grad():
        tl, tp_, tm = tiny(timgs, mask_ratio=0.6)
    data.update(tiny_imgs=timgs.numpy(), tiny_noise=tnoise.numpy(), tiny_loss=tl.numpy(), tiny_pred=tp_.numpy(),
                tiny_mask=tm.numpy())
    for k, v in tiny.state_dict().items():
        data["tiny_sd." + k] = v.numpy()
    np.savez_compressed(os.path.join(OUT, "mae_forward.npz"), **data)
    print("mae_forward.npz", float(loss), float(tl))


def gen_state_keys(MCM):
    """ordered state_dict keys + shapes of the default reference MCM (checkpoint compatibility)"""
    import json

    torch.manual_seed(0)
    ref = MCM(num_keep_patches=144)
    sd = ref.state_dict()
    init_sha = sha16(np.concatenate([v.float().numpy().ravel() for v in sd.values() if v.numel()]))
    with open(os.path.join(OUT, "mcm_state_keys.json"), "w") as f:
        json.dump({"keys": {k: list(v.shape) for k, v in sd.items()}, "init_sha_seed0": init_sha}, f)
    print("mcm_state_keys.json")


# ---------------------------------------------------------------------------------------- F3b
def gen_pos_interp():
    """interpolate_pos_embed (pos_embed.py:103-132, called by training.py:173-174 on --checkpoint): the
    reference function on seeded checkpoint tables, for target models given by (num_patches, rows of
    encoder_pos_embed) -- 14x14 -> 16x16 (224 checkpoint into a 256 model), 16x16 -> 12x12, same size"""
    import types

    from models.Compression.common.pos_embed import interpolate_pos_embed

    data = {}
    g = torch.Generator().manual_seed(21)
    for name, (src_g, dst_g, d, extra) in {"g14_to_g16": (14, 16, 96, 1), "g16_to_g12": (16, 12, 64, 1),
                                            "g8_to_g8": (8, 8, 32, 1), "g7_to_g9_two_extra": (7, 9, 16, 2)}.items():
        ck = {"pos_embed": torch.randn(1, extra + src_g * src_g, d, generator=g), "other": torch.zeros(1)}
        model = types.SimpleNamespace(encoder_embed=types.SimpleNamespace(num_patches=dst_g * dst_g),
                                      encoder_pos_embed=torch.zeros(1, extra + dst_g * dst_g, d))
        data[f"{name}_in"] = ck["pos_embed"].numpy()
        interpolate_pos_embed(model, ck)
        data[f"{name}_out"] = ck["pos_embed"].numpy()
        data[f"{name}_meta"] = np.array([src_g, dst_g, d, extra])
    np.savez_compressed(os.path.join(OUT, "pos_interp.npz"), **data)
    print("pos_interp.npz")


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", help="generators to run (default: all)")
    only = ap.parse_args().only
    os.makedirs(OUT, exist_ok=True)
    install_stubs()
    import models.Compression.common.pos_embed  # noqa: F401  (real reference module)
    from models.Compression.MCM import MCM

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    gens = {"ids": lambda: gen_ids(MCM), "pos": gen_pos, "pos_interp": gen_pos_interp,
            "tiny": lambda: gen_forward(MCM, "tiny", TINY, batch=2, seed=7),
            "small12": lambda: gen_forward(MCM, "small12", SMALL12, batch=2, seed=11),
            "mae_masking": gen_mae_masking, "mae_forward": gen_mae_forward, "state_keys": lambda: gen_state_keys(MCM)}
    for k, fn in gens.items():
        if not only or k in only:
            fn()


if __name__ == "__main__":
    main()
