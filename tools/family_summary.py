"""Per-forward kernel time by family from a rocprofv3 kernel trace (CSV), for cross-checking the
bench's live per-launch event timing (bench.py LaunchTimer).  Forwards are counted by the
ids-shuffle kernel (once per MCM forward).

Kernel name -> family (the shape -> family mapping of bench.py, by what the trace can tell apart):
  lic_conv3x3     conv_halo_kernel<...> and every GEMM tile with a ConvSrc operand source
  lic_latent      lic_latent_kernel<...> (the slice stacks' latent partial sums)
  enc_attn_core   mha_fwd_bf16_kernel<64>        dec_attn_core  mha_fwd_bf16_kernel<32>
  layernorm       layernorm_kernel
  gc_slices       gc_slices_kernel               eb_likelihood  eb_prep_kernel + eb_likelihood_kernel
  token_gemm      every other gemm_glds / gemm_reg / gemm_phased launch (qkv, proj, fc1, fc2, g_a, g_s,
                  patch embed, decoder embed / pred)
  other           entropy models, ids, copies

--replay: only the kernels after the last spin kernel, i.e. bench.py's family replays (1 warm-up + 5 timed
passes of each family's launches, back to back); the per-launch averages are what the bench line reports.
--forward: only the kernels before it (the bench's forwards: eager warm-ups, then the HIP-graph replays), per
forward as counted by the ids-shuffle kernel -- each kernel's duration inside the real forward.
--both: {"forward": ..., "replay": ...} in one file (profiles/rNN/trace_families.json, read by bench.py).

usage: python tools/family_summary.py <kernel_trace.csv> [--replay | --forward | --both] [--json out.json]
"""
import argparse
import csv
import json
from collections import defaultdict


def family(name):
    if "lic_stack_kernel" in name:
        return "lic_stack"
    if "lic_latent_kernel" in name:
        return "lic_latent"
    if "conv_halo_kernel" in name or ("gemm" in name and "ConvSrc" in name):
        return "lic_conv3x3"
    if "qkv_attn_kernel" in name:  # fused qkv GEMM + attention (bf16 inference): dh 64 encoder, dh 32 decoder
        return "enc_qkv_attn" if "qkv_attn_kernel<64," in name or "qkv_attn_kernelILi64E" in name else "dec_qkv_attn"
    if "mha_fwd" in name:
        return "enc_attn_core" if "<64>" in name or "ILi64E" in name else "dec_attn_core"
    if "layernorm_kernel" in name:
        return "layernorm"
    if "gc_slices_kernel" in name or "gc_slices_tiled_kernel" in name:
        return "gc_slices"
    if "eb_prep_kernel" in name or "eb_likelihood_kernel" in name:
        return "eb_likelihood"
    if "gemm_" in name:
        return "token_gemm"
    if "spin_kernel" in name:
        return None
    return "other"


def summarize(rows, mode):
    last = max((i for i, r in enumerate(rows) if "spin_kernel" in r["Kernel_Name"]), default=-1)
    if mode == "replay":
        rows = rows[last + 1:]
    elif mode == "forward" and last >= 0:
        rows = rows[:last]
    fam = defaultdict(lambda: [0, 0.0])
    halo = defaultdict(lambda: [0, 0.0])
    nfwd = 0
    for r in rows:
        n = r["Kernel_Name"]
        if "ids_shuffle" in n:
            nfwd += 1
        f = family(n)
        if f is None:
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        fam[f][0] += 1
        fam[f][1] += d
        if f == "lic_conv3x3":
            k = "conv_halo_kernel" if "conv_halo" in n else "gemm(ConvSrc)"
            halo[k][0] += 1
            halo[k][1] += d
    nfwd = 6 if mode == "replay" else max(nfwd, 1)  # replay mode: 1 warm-up + 5 timed passes
    return {"forwards": nfwd, "families": {k: {"launches_per_fwd": v[0] / nfwd, "us_per_fwd": round(v[1] / nfwd, 1),
                                                "avg_launch_us": round(v[1] / max(v[0], 1), 2)}
                                            for k, v in sorted(fam.items(), key=lambda kv: -kv[1][1])},
            "lic_conv3x3_split": {k: {"launches_per_fwd": v[0] / nfwd, "us_per_fwd": round(v[1] / nfwd, 1),
                                      "avg_launch_us": round(v[1] / max(v[0], 1), 2)} for k, v in halo.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--cite", default=None, help="the committed copy of the trace to name in the JSON (profiles/rNN/...)")
    ap.add_argument("--json")
    g = ap.add_mutually_exclusive_group()
    g.add_argument("--replay", action="store_true")
    g.add_argument("--forward", action="store_true")
    g.add_argument("--both", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.both:
        out = {"trace": a.cite or a.trace, "trace_raw": a.trace, "forward": summarize(rows, "forward"),
               "replay": summarize(rows, "replay")}
    else:
        out = summarize(rows, "replay" if a.replay else "forward" if a.forward else "all")
    print(json.dumps(out, indent=1))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
