#!/bin/bash
# round-2 call 27: fused stacks v6 (4 waves, strided output fragments, 8-step A ring)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_lstk:300:python -u -m pytest tests/test_gpu_lic_stack.py -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "lstk:200:python -u tools/lstk_bench.py" \
  "lstk_w0:200:TMAE_LSTK_FLAGS=0 python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "bench_new:200:$B" \
  "bench_old:200:TMAE_LIC_STACK=0 $B"
