"""Where a captured training step's time goes between kernels: from a rocprofv3 kernel trace (CSV) of graph replays,
take one whole step (between two relayout_multi launches), split its kernels into the compute chain and the
side streams (weight gradients gemm_tn / tn_reduce, RCCL), and print the HIP queues the compute chain ran on, every
queue hop with the idle gap in front of it, and the RCCL kernels.   python tools/graph_hops.py <kernel_trace.csv>"""
import csv
import sys

SIDE = ("gemm_tn", "tn_reduce", "oneRank")


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Queue_Id"])) for r in rows)
    starts = [k[0] for k in ks if "relayout_multi" in k[2]]
    a, b = starts[-2], starts[-1]
    st = [k for k in ks if a <= k[0] < b]
    comp = [k for k in st if not any(s in k[2] for s in SIDE)]
    rccl = [k for k in st if "oneRank" in k[2]]
    queues = sorted({k[3] for k in comp})
    hops = [(comp[i - 1], comp[i]) for i in range(1, len(comp)) if comp[i][3] != comp[i - 1][3]]
    gap = sum(max(0, n[0] - p[1]) for p, n in hops) / 1e3
    print(f"step span {(max(k[1] for k in st) - a) / 1e3:.0f} us (profiled), {len(st)} kernels; compute chain "
          f"{len(comp)} kernels on queues {queues}, {len(hops)} queue hops, {gap:.0f} us of idle gaps at the hops")
    for p, n in hops:
        print(f"  {(p[1] - a) / 1e3:9.1f} us  gap {max(0, n[0] - p[1]) / 1e3:7.1f} us  q{p[3]} -> q{n[3]}  "
              f"{p[2][:40]} -> {n[2][:40]}")
    for k in rccl:
        print(f"  RCCL {(k[0] - a) / 1e3:9.1f} us  {(k[1] - k[0]) / 1e3:6.1f} us  {k[2][:60]}")


if __name__ == "__main__":
    main(sys.argv[1])
