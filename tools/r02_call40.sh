#!/bin/bash
# round-2 call 40: LayerNorm with several rows per wave -- kernel tests, then bench A/B (rpw 4 / 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tests_kernels:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mcm.py tests/test_gpu_mae.py" \
  "bench_rpw:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_rpw1:400:TMAE_LN_RPW=1 python -u bench.py --no-train --no-cpu-baseline" \
  "bench_rpw2:400:python -u bench.py --no-train --no-cpu-baseline"
