#!/bin/bash
# Whole-forward A/B of the tile-choice efficiency knobs (gemm_core.h choose_tile): one bench process
# per setting, two interleaved repetitions.  usage: tools/ab_tiles.sh "ENV=V ENV2=V2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for e in "$@"; do
    v=$(env $e timeout -k 10 120 python bench.py --no-cpu-baseline --no-train --steps 40 2>/dev/null | tail -1 |
        python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$e -> $v"
  done
done
