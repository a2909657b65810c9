#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_conv:300:python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "conv_bench:200:python -u tools/conv_bench.py" \
  "bench1:200:$B" \
  "pytest_mcm:600:python -u -m pytest tests/test_gpu_mcm.py tests/test_gpu_bench_config.py -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "bench2:200:$B"
