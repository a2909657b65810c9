#!/bin/bash
# round-2 call 38: BASELINE config 4 bench line at HEAD (MCM with a ViT-L/16 encoder, batch 128)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "bench_cfg4:600:python -u bench.py --enc-dim 1024 --enc-depth 24 --enc-heads 16 --batch 128 --no-train --no-cpu-baseline"
