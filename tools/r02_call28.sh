#!/bin/bash
# round-2 call 28: forward with / without the lic_stack L2 warm-up, full bench line at HEAD, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "bench_w0:200:TMAE_LSTK_FLAGS=0 $B" \
  "bench_w1:200:TMAE_LSTK_FLAGS=1 $B" \
  "bench_w0b:200:TMAE_LSTK_FLAGS=0 $B" \
  "bench_w1b:200:TMAE_LSTK_FLAGS=1 $B" \
  "bench_full:600:python -u bench.py" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline"
