"""Summarise a rocprofv3 --stats kernel CSV: top kernels by total time, per-forward figures."""
import csv
import re
import sys

path = sys.argv[1]
nfwd = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms over the run; per forward ({nfwd:g}): {tot / 1e6 / nfwd:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    name = r["Name"]
    m = re.match(r"_Z\d+(\w+?)I(.*)", name)
    short = name if not m else m.group(1) + "<" + m.group(2)[:110]
    print(f"{float(r['TotalDurationNs']) / 1e6 / nfwd:8.3f} ms/fwd {float(r['Percentage']):6.2f}%  "
          f"calls/fwd {int(r['Calls']) / nfwd:6.1f}  avg {float(r['AverageNs']) / 1e3:8.1f} us  {short[:150]}")
