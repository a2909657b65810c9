#!/bin/bash
# round-2 call 32: forward kernel trace at HEAD (two-image halo conv default)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline"
