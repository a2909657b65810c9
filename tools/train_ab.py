"""A/B of training-step schedule hooks in ONE process on the same box: for each setting (class attributes of the
training executor, e.g. VIT_WG_SLOT_DIV), a fresh bench-config model, the graphed step (engine.GraphedTrainStep),
3 warm-up replays, N timed replays; prints ms per step for each setting, twice in alternating order.
    python tools/train_ab.py [steps] [batch] [setting ...]    setting = name=value[,name=value] or "base" """
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
import textmae_amd  # noqa: E402
from textmae_amd import engine, mcm_train  # noqa: E402
from textmae_amd.optim import configure_optimizers  # noqa: E402
from textmae_amd.rd_loss import RateDistortionLoss  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
settings = sys.argv[3:] or ["base"]
EAGER = "eager" in settings  # eager steps (engine.train_step) instead of the captured graph
settings = [st for st in settings if st != "eager"] or ["base"]


def parse(st):
    if st == "base":
        return {}
    return {k: int(v) for k, v in (kv.split("=") for kv in st.split(","))}


def run(st):
    saved = {k: getattr(mcm_train.TrainExec, k) for k in parse(st)}
    for k, v in parse(st).items():
        setattr(mcm_train.TrainExec, k, v)
    try:
        torch.manual_seed(0)
        m = textmae_amd.MCM(img_size=256, num_keep_patches=144).cuda().train()
        m.compute_dtype = torch.bfloat16
        m.distortion = "ssim+l1"
        opt, aux = configure_optimizers(m, lr=1e-4, aux_lr=1e-4, fused=True)
        crit = RateDistortionLoss(lmbda=1e-2)
        imgs, scores = bench.synthetic_inputs(B, 256, 256, 2000, "cuda")
        if EAGER:
            def g(i, s_):
                return engine.train_step(m, crit, i, s_, opt, aux, clip_max_norm=1.0)
        else:
            g = engine.GraphedTrainStep(m, crit, opt, aux, imgs, scores, clip_max_norm=1.0, warmup=1)
        for _ in range(3):
            g(imgs, scores)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g(imgs, scores)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / n * 1e3
        del g, m, opt, aux
        torch.cuda.empty_cache()
        return ms
    finally:
        for k, v in saved.items():
            setattr(mcm_train.TrainExec, k, v)


res = {st: [] for st in settings}
for rep in range(2):
    for st in (settings if rep == 0 else list(reversed(settings))):
        res[st].append(round(run(st), 3))
        print(st, res[st][-1], flush=True)
print(json.dumps({"batch": B, "steps": n, "eager": EAGER, "ms_per_step": res}))
