#!/bin/bash
# round-2 call 34: HEAD: full GPU suite, default bench line, kernel-trace profile, HBM traffic of the dominant
# family (lic_stack) from two PMC passes, smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --no-graph --steps 2 --warmup 1 --no-train --no-cpu-baseline --no-roofline"
bash tools/gpu_session.sh \
  "pytest_gpu:1100:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:600:python -u bench.py" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline" \
  "pmc_fetch:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o f -- $B" \
  "pmc_write:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o w -- $B"
