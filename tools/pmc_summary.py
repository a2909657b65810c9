"""Per-kernel mean of every counter in rocprofv3 --pmc counter_collection CSVs (one or more passes),
plus the derived fractions the stall analysis uses (SQ_* cycle counters are per-wave sums).

usage: python tools/pmc_summary.py <counter_collection.csv> [...] [--filter substr]
"""
import argparse
import csv
import re
from collections import defaultdict


def short(n):
    m = re.match(r"_Z\d+(\w+?)I(.*)", n)
    return (n if not m else m.group(1) + "<" + m.group(2))[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> dispatch -> value
    for path in a.csv:
        for r in csv.DictReader(open(path)):
            k = r.get("Kernel_Name", "")
            if a.filter and a.filter not in k:
                continue
            acc[short(k)][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, cs in acc.items():
        mean = {c: sum(d.values()) / max(1, len(d)) for c, d in cs.items()}
        n = max(len(d) for d in cs.values())
        print(f"== {k}  ({n} dispatches)")
        for c in sorted(mean):
            print(f"   {c:28s} {mean[c]:16.1f}")
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in mean:
                    print(f"   {c + ' / WAVE_CYCLES':40s} {mean[c] / wc:8.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in mean and "SQ_BUSY_CYCLES" in mean:
            print(f"   {'MFMA_BUSY / (BUSY x 4 SIMD x 256 CU)':40s} "
                  f"{mean['SQ_VALU_MFMA_BUSY_CYCLES'] / (mean['SQ_BUSY_CYCLES'] * 4 * 256):8.3f}")


if __name__ == "__main__":
    main()
