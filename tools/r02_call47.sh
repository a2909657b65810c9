#!/bin/bash
# round-2 call 47: final HEAD check (GPU suite, smoke, default bench line)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_gpu:1100:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:600:python -u bench.py"
