"""Per-stream view of one eager training step from a rocprofv3 kernel trace (tools/train_only.py under
`rocprofv3 --kernel-trace`): the last step is the span from the last-but-one adam_multi_kernel pair to the last one.
Prints, per queue/stream, the busy time and the kernel count; then the compute-queue kernels grouped into the
step's sections by name (forward, slice backward, ...), and the largest gaps on the compute queue.
    python tools/train_timeline.py <kernel_trace.csv>"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.match(r"_Z\d+(\w+?)I(.*)", n)
    n = n if not m else m.group(1) + "<" + m.group(2)
    return n[:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get(qkey, "?") if qkey else "?")
          for r in rows]
    ks.sort()
    adam = [i for i, k in enumerate(ks) if "adam_multi" in k[2]]
    # every step ends with two Adam launches (main + aux optimizer)
    ends = adam[1::2]
    if len(ends) < 2:
        print("need two steps in the trace")
        return
    a, b = ends[-2] + 1, ends[-1] + 1
    step = ks[a:b]
    t0, t1 = step[0][0], max(k[1] for k in step)
    print(f"step: {len(step)} kernels, span {(t1 - t0) / 1e3:.1f} us (columns: {qkey})")
    busy = defaultdict(float)
    cnt = defaultdict(int)
    for s, e, n, q in step:
        busy[q] += e - s
        cnt[q] += 1
    for q in sorted(busy, key=lambda q: -busy[q]):
        print(f"  queue {q}: {cnt[q]} kernels, busy {busy[q] / 1e3:.1f} us")
    main_q = max(cnt, key=lambda q: cnt[q])
    fam = defaultdict(lambda: [0, 0.0])
    for s, e, n, q in step:
        f = short(n)
        fam[(q, f)][0] += 1
        fam[(q, f)][1] += e - s
    print("top kernels per queue:")
    for (q, f), (c, t) in sorted(fam.items(), key=lambda x: -x[1][1])[:40]:
        print(f"  q{q} {t / 1e3:9.1f} us x{c:4d}  {f}")
    # union of busy intervals per queue vs the step span
    mq = sorted((s, e) for s, e, n, q in step if q == main_q)
    gaps = []
    cur = mq[0][1]
    for s, e in mq[1:]:
        if s > cur:
            gaps.append((s - cur, cur - t0))
        cur = max(cur, e)
    gaps.sort(reverse=True)
    print(f"main queue {main_q}: gaps total {sum(g for g, _ in gaps) / 1e3:.1f} us; largest:",
          ", ".join(f"{g / 1e3:.1f}us@{at / 1e3:.0f}" for g, at in gaps[:10]))


if __name__ == "__main__":
    main()
