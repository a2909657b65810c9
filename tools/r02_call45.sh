#!/bin/bash
# round-2 call 45: HEAD check after the lic_stack swap epilogue: full GPU suite, smoke, default bench line, kernel-trace
# profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_gpu:1100:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:600:python -u bench.py" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline"
