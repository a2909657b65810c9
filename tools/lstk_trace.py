"""Per-wave timeline of tmae_lic_stack from the LSTK_TRACE build (tools/build_variant.sh lstk_trace lic_stack.hip
-DLSTK_TRACE=1; run with TMAE_LIB=ab/libtmae_lstk_trace.so): for one eager launch of each shape, the shader-clock
stamps every wave wrote (lic_stack.hip g_lstk_trace) folded into, per layer, the mean / max over workgroups of
  span   = last wave done - first wave start (the layer's critical path),
  K      = K-loop cycles of the busiest wave (its items' MFMA loops), Kavg its mean over the 8 waves,
  E      = epilogue cycles of the busiest wave, Eavg,
  idle   = mean cycles a wave waits at the layer barrier (done -> next layer start),
plus the prologue (layer-0 input to LDS) and the launch's HIP-event time.  Shapes as tools/lstk_bench.py, and
`chain_3` = the forward's chained launch of serial slice 3 (mean + scale stacks, the mean stack going on into the
lrp stack).   usage: TMAE_LIB=... python tools/lstk_trace.py [shape ...]"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import _lib, ops  # noqa: E402

MID = [224, 176, 128, 80, 32]
SHAPES = {"ms_3": (96, 0, 2, 1), "lrp_3": (128, 0, 1, 1), "b_ms": (192, 0, 2, 6), "b_lrp": (192, 32, 1, 6)}
NWG, SLOTS = 1024, 48


def read_trace():
    lib = _lib.load()
    buf = np.zeros(NWG * 8 * SLOTS, dtype=np.uint64)
    if lib.tmae_lstk_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes)) != 0:
        raise RuntimeError("trace read failed")
    return buf.reshape(NWG, 8, SLOTS).astype(np.int64)


def analyse(tr, nwg, nlayers):
    tr = tr[:nwg]
    t0 = tr[:, :, 0].min(axis=1, keepdims=True)
    rel = tr - t0[:, :, None]
    out = {"wgs": nwg, "wg_cycles_mean": float((tr[:, :, 47].max(1) - t0[:, 0]).mean()),
           "prologue_cycles_mean": float((rel[:, :, 1]).mean())}
    layers = []
    for l in range(nlayers):
        b = 2 + 4 * l
        start, k, e, done = rel[:, :, b], tr[:, :, b + 1], tr[:, :, b + 2], rel[:, :, b + 3]
        nxt = rel[:, :, b + 4] if l + 1 < nlayers else rel[:, :, 47]
        span = done.max(1) - start.min(1)
        layers.append({"l": l, "span": int(span.mean()), "span_max": int(span.max()),
                       "K": int(k.max(1).mean()), "Kavg": int(k.mean()), "E": int(e.max(1).mean()),
                       "Eavg": int(e.mean()), "idle": int((nxt - done).mean()),
                       "barrier_skew": int((start.max(1) - start.min(1)).mean())})
    out["layers"] = layers
    return out


def main():
    lib = _lib.load()
    if not hasattr(lib, "tmae_lstk_trace_read"):
        raise SystemExit("not an LSTK_TRACE build: set TMAE_LIB=ab/libtmae_lstk_trace.so")
    names = sys.argv[1:] or ["ms_3", "chain_3", "lrp_3", "b_ms", "b_lrp"]
    B, G = 64, 12
    rows = B * G * G
    torch.manual_seed(0)
    res = {}
    for name in names:
        chain = name.startswith("chain")
        c1, c2, nb1, nb2 = SHAPES["ms_3" if chain else name]
        P = nb1 * nb2
        x1 = torch.randn(rows, 384, device="cuda").to(torch.bfloat16)
        chans = [c1 + c2] + MID

        def stackw(cin0, P):
            ch = [cin0] + MID
            return [torch.stack([ops.pack_lic_stack_weight(torch.randn(ch[l + 1], ch[l], 3, 3, device="cuda")
                                                           / (3 * max(ch[l], 1) ** 0.5)) for _ in range(P)])
                    for l in range(5)]
        ws = stackw(chans[0], P)
        bs = [torch.randn(P, c, device="cuda") * 0.1 for c in MID]
        add = torch.randn(rows, 8064, device="cuda")
        y = torch.empty(P, rows, 32, device="cuda")
        src = torch.randn(rows, 384, device="cuda")
        yb = torch.empty(rows, 384, device="cuda", dtype=torch.bfloat16)
        st = {"a": (224 * nb2, 224), "y": (nb2 * rows * 32, rows * 32), "x2": (0, 32), "src": (0, 32)}
        for l in range(5):
            st[f"w{l}"] = (nb2 * ws[l][0].numel(), ws[l][0].numel())
            st[f"b{l}"] = (nb2 * MID[l], MID[l])
        lrp = name.endswith("lrp") or name.startswith("lrp")
        kw = {}
        if chain:  # the slice's lrp stack (input 96 + 32 channels) after the mean stack, in the same workgroup
            lw = stackw(128, 1)
            kw = dict(chain=dict(w=[w[0] for w in lw], b=[torch.randn(c, device="cuda") * 0.1 for c in MID],
                                 couts=MID, x1=x1, c1=96, ld1=384, y=src, ldy=384, ypre=torch.empty_like(src),
                                 ld_ypre=384, add=add, ld_add=8064, out=yb, ld_out=384))

        def run():
            if lrp:
                st["y"] = (0, 32)
                ops.lic_stack(B, G, x1, c1, 384, ws, bs, MID, yb, 384, False, x2=x1 if c2 else None, c2=c2, ld2=384,
                              addend=add, ld_add=8064, lrp_src=src, ld_src=384, nb=(nb1, nb2), strides=st)
            else:
                ops.lic_stack(B, G, x1, c1, 384, ws, bs, MID, y, 32, True, addend=add, ld_add=8064, nb=(nb1, nb2),
                              strides=st, **kw)

        for _ in range(3):
            run()
        torch.cuda.synchronize()
        if lib.tmae_lstk_trace_reset() != 0:
            raise RuntimeError("trace reset failed")
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        e.synchronize()
        tr = read_trace()
        tr = tr[:min(P * B, NWG)]
        if chain:  # mean-stack workgroups run 10 layers (mean + lrp), scale-stack ones 5
            long_ = tr[:, 0, 2 + 4 * 5] != 0
            r = {"mean+lrp": analyse(tr[long_], int(long_.sum()), 10),
                 "scale": analyse(tr[~long_], int((~long_).sum()), 5)}
        else:
            r = analyse(tr, len(tr), 5)
        r["event_us"] = round(s.elapsed_time(e) * 1e3, 1)
        res[name] = r
        print(name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
