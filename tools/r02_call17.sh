#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_train:600:python -u -m pytest tests/test_gpu_train.py -q --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "train_wall:300:python -u tools/train_only.py 5" \
  "train_wall2:300:python -u tools/train_only.py 5" \
  "dump:300:python -u bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --dump-launches gpurun_out/launch_families.json"
