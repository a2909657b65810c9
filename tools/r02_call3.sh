#!/bin/bash
# round-2 call 3: new eval / score / DP tests, bench + kernel trace (replay agreement)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_new:600:python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_optim_dp.py -v -s --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-train --no-cpu-baseline"
