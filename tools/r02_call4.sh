#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_vgg:400:python -u -m pytest tests/test_gpu_vgg.py -v -s --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "pytest_all:1200:python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider"
