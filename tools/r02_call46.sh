#!/bin/bash
# round-2 call 46: decoder attention (dh = 32) with two 32-query blocks per wave (TMAE_MHA_QB=2: 5-wave
# workgroups, three per CU) vs one -- mha tests under both, bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "tests_qb2:300:TMAE_MHA_QB=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_mcm.py tests/test_gpu_bench_config.py" \
  "tests_qb1:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k mha" \
  "bench_qb1:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_qb2:400:TMAE_MHA_QB=2 python -u bench.py --no-train --no-cpu-baseline" \
  "bench_qb1b:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_qb2b:400:TMAE_MHA_QB=2 python -u bench.py --no-train --no-cpu-baseline"
