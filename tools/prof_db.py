"""Summarise a rocprofv3 rocpd database (kernel trace): per-kernel (and per launch grid) time per
forward.  Forwards are counted by the ids-shuffle kernel, which runs once per MCM forward.

usage: python tools/prof_db.py <run_results.db> [top] [--by-grid] [--csv out.csv]
"""
import argparse
import csv
import re
import sqlite3


def short(name):
    m = re.match(r"_Z\d+(\w+?)I(.*)", name)
    return name if not m else m.group(1) + "<" + m.group(2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("top", nargs="?", type=int, default=30)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--csv")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, grid_x, grid_y, workgroup_x, duration from kernels").fetchall()
    nfwd = sum(1 for r in rows if "ids_shuffle" in r[0]) or 1
    agg = {}
    for name, gx, gy, wx, dur in rows:
        key = (name, f"{gx // max(wx, 1)}x{gy}") if a.by_grid else (name, "")
        t = agg.setdefault(key, [0, 0.0])
        t[0] += 1
        t[1] += dur
    tot = sum(v[1] for v in agg.values())
    print(f"{len(rows)} dispatches, {nfwd} forwards; kernel time per forward {tot / nfwd / 1e6:.3f} ms")
    out = []
    for (name, grid), (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out.append({"name": name, "grid": grid, "calls_per_fwd": n / nfwd, "avg_us": d / n / 1e3,
                    "ms_per_fwd": d / nfwd / 1e6, "pct": 100.0 * d / tot})
    for r in out[:a.top]:
        print(f"{r['ms_per_fwd']:7.3f} ms {r['pct']:5.1f}%  x{r['calls_per_fwd']:5.1f}  avg {r['avg_us']:8.1f} us "
              f"{r['grid']:>9} {short(r['name'])[:130]}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(out[0]))
            w.writeheader()
            w.writerows(out)


if __name__ == "__main__":
    main()
