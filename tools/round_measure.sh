#!/bin/bash
# The round's evidence pass at HEAD, one gpurun call: the full GPU suite (fresh parity log), smoke, the
# default bench line, the forward kernel trace (trace_families.json), the two PMC passes
# (pmc_families.json), the config-4 line and a training kernel profile.  Outputs under gpurun_out/<tag>_*;
# copy what DESIGN.md cites into profiles/rNN/.   usage: tools/round_measure.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-m}
rm -f gpurun_out/parity_metrics.jsonl
tools/gpu_session.sh \
  "${tag}_pytest:900:python -u -m pytest tests -m gpu -q -rf --timeout 170 --timeout-method thread" \
  "${tag}_smoke:300:python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "${tag}_bench:500:python bench.py" \
  "${tag}_trace:400:tools/trace_bench.sh $tag" \
  "${tag}_pmc:600:tools/pmc_bench.sh $tag lic_stack" \
  "${tag}_cfg4:400:python bench.py --enc-dim 1024 --enc-depth 24 --enc-heads 16 --batch 128 --no-cpu-baseline --no-train --no-k64 --no-distortion" \
  "${tag}_maelarge:300:python bench.py --mae-large --no-cpu-baseline --no-train --no-k64 --no-distortion --no-roofline --no-mae-train" \
  "${tag}_proftrain:400:rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${tag}_ptrain -o t -- python3 bench.py --no-cpu-baseline --no-k64 --no-roofline --no-distortion --no-dp-rehearsal --no-mae-train --steps 3 --warmup 1" || exit $?
cp "$(find gpurun_out/${tag}_ptrain -name '*kernel_stats.csv' | head -1)" "gpurun_out/${tag}_train_kernel_stats.csv"
kt=$(find "gpurun_out/trace_${tag}" -name '*kernel_trace.csv' | head -1)
python3 tools/fwd_trace.py "$kt" > "gpurun_out/${tag}_fwd_timeline.txt"
python3 tools/fwd_trace.py "$kt" --sum > "gpurun_out/${tag}_fwd_timeline_sum.txt"
rm -rf "gpurun_out/${tag}_ptrain" "gpurun_out/trace_${tag}" gpurun_out/pmc_${tag}_*
cp gpurun_out/parity_metrics.jsonl "gpurun_out/${tag}_parity_metrics.jsonl"
echo "measure $tag done"
