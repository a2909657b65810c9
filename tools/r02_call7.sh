#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_train:600:python -u -m pytest tests/test_gpu_train.py tests/test_gpu_optim_dp.py -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "train_wall:300:python -u tools/train_only.py 5" \
  "train_prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o t -f csv -- python3 tools/train_only.py 3"
