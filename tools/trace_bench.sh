#!/bin/bash
# rocprofv3 kernel trace (+ --stats) of the bench's forward section and its family replays, then the
# per-family summary (tools/family_summary.py --both) that bench.py reads as profiles/rNN/trace_families.json.
# usage: tools/trace_bench.sh <tag> [extra bench.py args]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/trace_$tag
rm -rf "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$out" -o bench -- \
  python3 bench.py --no-cpu-baseline --no-train --no-k64 --no-distortion --no-mae-train "$@" > "gpurun_out/trace_${tag}_bench.json"
kt=$(find "$out" -name '*kernel_trace.csv' | head -1)
ks=$(find "$out" -name '*kernel_stats.csv' | head -1)
# a compact copy of the raw trace (name, queue, start / end ns, grid, workgroup) to commit beside the summary it backs
python3 - "$kt" "gpurun_out/kernel_trace_${tag}.csv" <<'PY'
import csv, sys
cols = ["Kernel_Name", "Queue_Id", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X",
        "LDS_Block_Size", "VGPR_Count"]
with open(sys.argv[1]) as f, open(sys.argv[2], "w", newline="") as g:
    w = csv.writer(g)
    w.writerow(cols)
    for r in csv.DictReader(f):
        w.writerow([r[c] for c in cols])
PY
gzip -f "gpurun_out/kernel_trace_${tag}.csv"
python3 tools/family_summary.py "$kt" --both --json "gpurun_out/trace_families_${tag}.json" --cite "${PROFILE_DIR:-profiles/r06}/kernel_trace_${tag}.csv.gz" > /dev/null
cp "$ks" "gpurun_out/kernel_stats_${tag}.csv"
echo "trace $tag: $kt"
