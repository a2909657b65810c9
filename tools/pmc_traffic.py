"""HBM traffic of the roofline kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md § HBM):
FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), FETCH_SIZE doubled on gfx950 (128-B
requests tallied at 64 B), WRITE_SIZE exact for 16-B-per-lane stores.  Both counters are in KiB.

usage: python tools/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, counter, kernel_sub="gemm"):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") == counter and kernel_sub in r.get("Kernel_Name", ""):
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(vals.values())
    return v[len(v) // 2] if v else None, len(v)


def main():
    fetch, nf = per_dispatch(sys.argv[1], "FETCH_SIZE")
    write, nw = per_dispatch(sys.argv[2], "WRITE_SIZE")
    M, N, K = 64 * 145, 3072, 768
    alg = (M * K + N * K + M * N) * 2 + N * 4
    out = {"kernel": "enc fc1+GELU GEMM (M=9280,N=3072,K=768,bf16)", "dispatches": [nf, nw],
           "fetch_kib_raw_median": fetch, "write_kib_median": write,
           "hbm_bytes_per_launch": int((2 * fetch + write) * 1024) if fetch is not None and write is not None else None,
           "algorithmic_bytes_per_launch": alg,
           "note": "FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE; median over dispatches; Infinity-Cache hits "
                   "are counted as fetches by these counters"}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
