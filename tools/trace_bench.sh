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
python3 tools/family_summary.py "$kt" --both --json "gpurun_out/trace_families_${tag}.json" > /dev/null
cp "$ks" "gpurun_out/kernel_stats_${tag}.csv"
echo "trace $tag: $kt"
