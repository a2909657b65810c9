"""Workgroup timeline of gemm_glds_kernel from the TMAE_GEMM_TRACE build (tools/build_variant.sh gemm_trace gemm.hip
-DTMAE_GEMM_TRACE=1; run with TMAE_LIB=ab/libtmae_gemm_trace.so).  One eager launch per token-GEMM shape of
tools/gemm_bench.py after warm-up; wave 0 of every workgroup stamped (s_memtime, shader clock) its start, the
prologue's DMA wait, the end of its K loop, the end of its epilogue's issue and the completion of its stores.
Per shape: mean cycles of prologue / K loop / epilogue issue / store drain, the launch span per XCC (its clock), and
how many workgroups sit in each phase over time (8 time bins of the span): with every workgroup of a round in its
epilogue at once the MFMA pipes idle while the stores drain.   usage: TMAE_LIB=... python tools/gemm_trace.py [shape]"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import textmae_amd  # noqa: E402,F401
from textmae_amd import _lib, ops  # noqa: E402
from gemm_bench import SHAPES  # noqa: E402

NWG, SLOTS = 8192, 8


def main():
    lib = _lib.load()
    if not hasattr(lib, "tmae_gemm_trace_read"):
        raise SystemExit("not a TMAE_GEMM_TRACE build")
    dt = torch.bfloat16
    torch.manual_seed(0)
    for name in sys.argv[1:] or ["enc_fc1", "enc_fc1_noact", "enc_qkv", "enc_fc2", "enc_proj", "dec_fc1"]:
        M, N, K, act = SHAPES[name]
        x = torch.randn(M, K, device="cuda").to(dt)
        w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(dt)
        b = torch.randn(N, device="cuda")
        y = torch.empty(M, N, device="cuda", dtype=dt)
        for _ in range(3):
            ops.linear(x, w, b, dt, act=act, out=y)
        torch.cuda.synchronize()
        if lib.tmae_gemm_trace_reset() != 0:
            raise RuntimeError("trace reset failed")
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        ops.linear(x, w, b, dt, act=act, out=y)
        e.record()
        e.synchronize()
        buf = np.zeros(NWG * SLOTS, dtype=np.uint64)
        lib.tmae_gemm_trace_read(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
        tr = buf.reshape(NWG, SLOTS).astype(np.int64)
        tr = tr[tr[:, 0] != 0]
        xcc = tr[:, 5] & 0xF
        r = {"wgs": len(tr), "event_us": round(s.elapsed_time(e) * 1e3, 1)}
        r["prologue"] = int((tr[:, 1] - tr[:, 0]).mean())
        r["kloop"] = int((tr[:, 2] - tr[:, 1]).mean())
        r["epi_issue"] = int((tr[:, 3] - tr[:, 2]).mean())
        r["store_drain"] = int((tr[:, 6] - tr[:, 3]).mean())
        spans, phases = [], np.zeros((8, 4))
        for c in np.unique(xcc):
            t = tr[xcc == c]
            t0, t1 = t[:, 0].min(), t[:, 6].max()
            spans.append(int(t1 - t0))
            # phase occupancy: workgroups in prologue / K loop / epilogue issue / store drain per time bin
            edges = np.linspace(t0, t1, 9)
            for bi in range(8):
                mid = (edges[bi] + edges[bi + 1]) / 2
                for ph in range(4):
                    a, bcol = [(0, 1), (1, 2), (2, 3), (3, 6)][ph]
                    phases[bi, ph] += ((t[:, a] <= mid) & (mid < t[:, bcol])).sum()
        r["span_cycles_per_xcc"] = spans
        r["cycles_per_us"] = round(np.mean(spans) / max(r["event_us"], 1e-9), 1)
        r["phase_occupancy_per_bin(pro,k,epi,drain)"] = (phases / len(np.unique(xcc))).round(1).tolist()
        print(name, json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
