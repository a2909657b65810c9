"""HBM traffic per kernel family from two rocprofv3 PMC passes (MI355X_MICROARCH.md § HBM): FETCH_SIZE
and WRITE_SIZE in separate passes, FETCH_SIZE doubled (gfx950 tallies 128-B requests at 64 B), WRITE_SIZE
as read; both counters in KiB.  Forwards are counted by the ids-shuffle dispatches; families as in
tools/family_summary.py.

usage: python tools/pmc_family.py <fetch counter_collection.csv> <write counter_collection.csv> <family> [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from family_summary import family  # noqa: E402


def per_family(path, counter):
    disp = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        disp[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
        names[int(r["Dispatch_Id"])] = r["Kernel_Name"]
    # tools/fwd_only.py runs whole forwards and nothing else: the first one (weight init and re-layout, workspace
    # set-up) is a warm-up, so counting starts at the SECOND forward's ids_shuffle dispatch
    starts = sorted(d for d, n in names.items() if "ids_shuffle" in n)
    first = starts[1] if len(starts) > 1 else (starts[0] if starts else 0)
    disp = {d: v for d, v in disp.items() if d >= first}
    fwd = max(len(starts) - 1, 1)
    fam = defaultdict(lambda: [0, 0.0])
    for d, v in disp.items():
        f = family(names[d])
        if f is None:
            continue
        fam[f][0] += 1
        fam[f][1] += v
    return fam, fwd


def main():
    fetch, nf = per_family(sys.argv[1], "FETCH_SIZE")
    write, nw = per_family(sys.argv[2], "WRITE_SIZE")
    fam = sys.argv[3]
    out = {"family": fam, "forwards": [nf, nw], "per_family": {}}
    for f in sorted(set(fetch) | set(write)):
        n = max(fetch[f][0], 1)
        byts = (2 * fetch[f][1] + write[f][1]) * 1024
        # the profiled run holds only whole forwards (tools/pmc_bench.sh: --no-roofline, no replays), so a
        # family's launches per forward = its launches / forwards, and per-forward bytes = per-launch bytes x that
        lpf = fetch[f][0] / nf
        out["per_family"][f] = {"launches": fetch[f][0], "launches_per_fwd": round(lpf, 3),
                                "fetch_kib_raw": round(fetch[f][1], 1), "write_kib": round(write[f][1], 1),
                                "hbm_bytes_per_launch": int(byts / n), "hbm_bytes_per_fwd": int(byts / n * lpf)}
    d = out["per_family"].get(fam)
    out["hbm_bytes_per_launch"] = d["hbm_bytes_per_launch"] if d else None
    out["note"] = ("FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, summed over the family's dispatches of a run of "
                   "whole eager forwards and nothing else (tools/fwd_only.py; dispatches before the first ids_shuffle "
                   "dropped), divided by its launch count; Infinity-Cache hits are counted as fetches by these counters")
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
