#!/bin/bash
# round-2 call 33: chained serial slices (mean stack -> y_hat_pre -> lrp stack per launch, likelihoods deferred)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_lstk:400:python -u -m pytest tests/test_gpu_lic_stack.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider" \
  "bench_c1:200:TMAE_LIC_CHAIN=1 $B" \
  "bench_c0:200:TMAE_LIC_CHAIN=0 $B" \
  "bench_c1b:200:TMAE_LIC_CHAIN=1 $B" \
  "bench_c0b:200:TMAE_LIC_CHAIN=0 $B" \
  "bench_cb:200:TMAE_LIC_CHAIN_B=1 $B" \
  "bench_cbb:200:TMAE_LIC_CHAIN_B=1 $B" \
  "pytest_more:900:python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_coding.py tests/test_gpu_mcm.py tests/test_gpu_eval.py -q --timeout 300 --timeout-method thread -p no:cacheprovider"
