"""Per-kernel SQ stall breakdown from a rocprofv3 --pmc counter_collection.csv (tools/gemm_pmc.sh).

For each kernel name (dispatches summed): the share of wave cycles parked in s_waitcnt / s_barrier (WAIT_ANY),
issue-stalled (WAIT_INST_ANY, of which LDS issue WAIT_INST_LDS) and issuing (ACTIVE_INST_ANY); the MFMA pipe's
busy share of the kernel's CU cycles; LDS bank-conflict cycles over all LDS-array cycles; the effective clock.
SQ_WAVE_CYCLES / WAIT / ACTIVE count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE count cycles
(MI355X_MICROARCH.md, per-instruction table and DVFS note).

usage: python tools/sq_summary.py <counter_collection.csv | results.db>
"""
import csv
import sys
from collections import defaultdict


def main(path):
    per = defaultdict(lambda: defaultdict(float))
    ndisp = defaultdict(set)
    dur = {}
    if path.endswith(".db"):  # rocprofv3's default rocpd output
        import sqlite3

        rows = sqlite3.connect(path).execute(
            "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection")
        recs = ((str(d), k, c, v, t) for d, k, c, v, t in rows)
    else:
        recs = ((r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]),
                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(path)))
    for did, name, cname, val, d in recs:
        per[name][cname] += float(val)
        ndisp[name].add(did)
        dur[(name, did)] = d
    rows = []
    for name, c in per.items():
        wc = c["SQ_WAVE_CYCLES"] or 1.0
        n = len(ndisp[name])
        ns = sum(v for (k, _), v in dur.items() if k == name) / max(n, 1)
        gui = c["GRBM_GUI_ACTIVE"] / n if n else 0.0
        clk = gui / 8 / ns if ns else 0.0  # GHz: summed over 8 XCDs
        busy_cu = c["SQ_VALU_MFMA_BUSY_CYCLES"] / n / (256 * 4) if n else 0.0  # per SIMD
        mfma_util = busy_cu / (gui / 8) if gui else 0.0
        rows.append((c["SQ_WAVE_CYCLES"], name, n, c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc,
                     c["SQ_WAIT_INST_LDS"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc, mfma_util,
                     c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1.0), ns / 1e3, clk))
    print(f"{'disp':>4} {'us':>7} {'GHz':>5} {'wait':>5} {'istall':>6} {'lds_is':>6} {'active':>6} {'mfma':>5} "
          f"{'bankc':>5}  kernel")
    for _, name, n, wa, wi, wl, ac, mu, bc, us, clk in sorted(rows, reverse=True):
        print(f"{n:4d} {us:7.1f} {clk:5.2f} {wa:5.2f} {wi:6.2f} {wl:6.2f} {ac:6.2f} {mu:5.2f} {bc:5.2f}  {name[:150]}")


if __name__ == "__main__":
    main(sys.argv[1])
