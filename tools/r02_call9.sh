#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "conv_pf0:200:TMAE_CONV_PREFETCH=0 python -u tools/conv_bench.py" \
  "conv_pf8:200:TMAE_CONV_PREFETCH=8 python -u tools/conv_bench.py" \
  "conv_pf2:200:TMAE_CONV_PREFETCH=2 python -u tools/conv_bench.py" \
  "pytest_mha:300:python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -q -k 'mha' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "attn_bench:200:python -u tools/attn_bench.py" \
  "pytest_conv:300:python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "bench_pf0:200:TMAE_CONV_PREFETCH=0 $B" \
  "bench_pf8:200:TMAE_CONV_PREFETCH=8 $B" \
  "bench_pf0b:200:TMAE_CONV_PREFETCH=0 $B" \
  "bench_pf8b:200:TMAE_CONV_PREFETCH=8 $B"
