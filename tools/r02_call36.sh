#!/bin/bash
# round-2 call 36: serial-slice likelihoods on the side stream (TMAE_LIC_SIDE_LIK) A/B + tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_lstk:400:python -u -m pytest tests/test_gpu_lic_stack.py tests/test_gpu_bench_config.py -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench_s1:200:TMAE_LIC_SIDE_LIK=1 $B" \
  "bench_s0:200:TMAE_LIC_SIDE_LIK=0 $B" \
  "bench_s1b:200:TMAE_LIC_SIDE_LIK=1 $B" \
  "bench_s0b:200:TMAE_LIC_SIDE_LIK=0 $B"
