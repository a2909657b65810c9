"""Print the kernel timeline of one MCM forward from a rocprofv3 kernel trace (CSV or rocpd .db): the
launches between two consecutive ids_shuffle dispatches, with start offset, duration, grid,
registers and LDS.  --sum prints per-section totals instead (encoder / LIC / decoder by position).

usage: python tools/fwd_trace.py <kernel_trace.csv | results.db> [--which -2] [--sum]
"""
import argparse
import csv
import re
import sqlite3


def short(n):
    m = re.match(r"_Z\d+(\w+?)I(.*)", n)
    n = n if not m else m.group(1) + "<" + m.group(2)
    return n[:110]


def load(path):
    """rows of (name, start, end, grid_wg, grid_y, vgpr, agpr, lds) in dispatch order"""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        q = ("select name, start, end, grid_x / max(workgroup_x, 1), grid_y, vgpr_count, accum_vgpr_count, lds_size "
             "from kernels order by start")
        return [tuple(r) for r in c.execute(q)]
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Grid_Size_Y"]),
                    int(r["VGPR_Count"]), int(r["Accum_VGPR_Count"]), int(r["LDS_Block_Size"])))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--which", type=int, default=-2)
    ap.add_argument("--sum", action="store_true")
    a = ap.parse_args()
    rows = load(a.trace)
    idx = [i for i, r in enumerate(rows) if "ids_shuffle" in r[0]]
    lo, hi = idx[a.which], idx[a.which + 1]
    t0 = rows[lo][1]
    tot = gaps = 0.0
    prev_end = None
    agg = {}
    for name, s, e, g, gy, vg, ag, lds in rows[lo:hi]:
        d = (e - s) / 1e3
        tot += d
        if prev_end:
            gaps += max(0, s - prev_end) / 1e3
        prev_end = e
        k = short(name)[:60]
        agg.setdefault(k, [0, 0.0])
        agg[k][0] += 1
        agg[k][1] += d
        if not a.sum:
            print(f"{(s - t0) / 1e3:8.1f} {d:7.1f} us  wg={g:5d}x{gy:>3} vgpr={vg:>3}/{ag:>3} lds={lds:>6}  {short(name)}")
    if a.sum:
        for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            print(f"{d:8.1f} us  x{n:3d}  {k}")
    print("kernel sum %.1f us, gaps %.1f us, span %.1f us" % (tot, gaps, (rows[hi][1] - t0) / 1e3))


if __name__ == "__main__":
    main()
