#!/bin/bash
# round-2 call 16: training tests at HEAD, the default bench line, a kernel-trace profile of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_train:600:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_optim_dp.py tests/test_gpu_vgg.py -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "bench:600:python -u bench.py" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-train --no-cpu-baseline" \
  "train_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o t -f csv -- python3 tools/train_only.py 3"
