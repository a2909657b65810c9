"""Per-mode timing of the training step's weight re-layout (mcm_train._Weights.refresh -> tmae_relayout_multi) at
the bench config (ViT-B MCM, batch 64, bf16): one eager step fills the cache, then each group of entries (all, and
each relayout mode alone) is marked stale and re-laid out; GPU time from events around the launch (a sleep kernel
ahead of it hides the host's table work), bytes = f32 source read + destination written.
    python tools/relayout_bench.py"""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine  # noqa: E402
from textmae_amd.mcm_train import _Weights  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402


def mode_of(job):
    if job[0] == "licT":
        return "m4_licT"
    if job[0] == "lic":
        return "m3_lic"
    dims, strides = job
    d = list(dims) + [1] * (4 - len(dims))
    st = list(strides) + [0] * (4 - len(strides))
    if _Weights._is_transpose(dims, strides):
        return "m1_transpose"
    if d[1] * d[2] * d[3] <= 8192 and st[2] == 1 and st[1] == d[2] and st[3] == d[1] * d[2] and st[0] == d[1] * d[2] * d[3]:
        return "m2_rows"
    return "m0_cast"


def main():
    torch.manual_seed(0)
    m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
    m.compute_dtype = torch.bfloat16
    m.distortion = "ssim+l1"
    opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
    crit = RateDistortionLoss(lmbda=1e-2)
    imgs, scores = bench.synthetic_inputs(64, 256, 256, 2000, "cuda")
    engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
    engine.train_step(m, crit, imgs, scores, opt, aux, clip_max_norm=1.0)
    torch.cuda.synchronize()
    W = m._train_exec.w
    entries = [e for e in W.cache.values() if e[3] is not None]
    groups = {"all": entries}
    for e in entries:
        groups.setdefault(mode_of(e[3]), []).append(e)
    res = {}
    for name, ents in groups.items():
        nbytes = sum(e[1].numel() * e[1].element_size() for e in ents)
        src = 0
        for e in ents:  # f32 bytes the entry reads
            job = e[3]
            if job[0] == "lic":
                src += 4 * 9 * job[1] * job[4]
            elif job[0] == "licT":
                src += 4 * 9 * job[1] * job[2]
            else:
                src += 4 * e[1].numel()
        best = 1e9
        for rep in range(6):
            for e in ents:
                e[0] = (0, 0)
            torch.cuda.synchronize()
            torch.cuda._sleep(50_000_000)
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            W.refresh()
            t.record()
            t.synchronize()
            if rep:
                best = min(best, s.elapsed_time(t) * 1e3)
        res[name] = {"entries": len(ents), "us": round(best, 1), "dst_MB": round(nbytes / 1e6, 1),
                     "src_MB": round(src / 1e6, 1), "GB_s": round((nbytes + src) / best / 1e3, 1)}
        print(name, res[name], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
