#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_conv3:300:TMAE_CONV_TPS=3 python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "conv_t1:200:TMAE_CONV_TPS=1 python -u tools/conv_bench.py" \
  "conv_t3:200:TMAE_CONV_TPS=3 python -u tools/conv_bench.py" \
  "bench_t1:200:TMAE_CONV_TPS=1 $B" \
  "bench_t3:200:TMAE_CONV_TPS=3 $B" \
  "bench_t1b:200:TMAE_CONV_TPS=1 $B" \
  "bench_t3b:200:TMAE_CONV_TPS=3 $B"
