#!/bin/bash
# round-2 call 41: 3-stage ring for 64x128 GEMM tiles added to the deep ring -- kernel tests, then bench A/B (deep on / off)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tests_kernels:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mcm.py" \
  "bench_deep:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_flat:400:TMAE_GEMM_DEEP=0 python -u bench.py --no-train --no-cpu-baseline" \
  "bench_deep2:400:python -u bench.py --no-train --no-cpu-baseline"
