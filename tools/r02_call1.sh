#!/bin/bash
# round-2 GPU call: full GPU suite, default bench line, config-4 bench line, kernel-trace profile of the bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest:1000:python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "bench:400:python -u bench.py > gpurun_out/bench.json" \
  "bench_cfg4:400:python -u bench.py --enc-dim 1024 --enc-depth 24 --enc-heads 16 --batch 128 --no-train --no-cpu-baseline > gpurun_out/bench_cfg4.json" \
  "prof:400:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 10 --warmup 2 --no-train --no-cpu-baseline"
