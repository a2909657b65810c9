#!/bin/bash
# round-2 call 35: default bench line (chain-aware lic_stack FLOP accounting) twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "bench:600:python -u bench.py" \
  "bench2:300:python -u bench.py --no-train --no-cpu-baseline"
