#!/bin/bash
# round-2 call 19: fused slice stacks v2 (two output fragments per item, conflict-free pitch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_lstk:300:python -u -m pytest tests/test_gpu_lic_stack.py -v -s --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bench_new:200:$B" \
  "bench_old:200:TMAE_LIC_STACK=0 $B" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline"
