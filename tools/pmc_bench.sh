#!/bin/bash
# HBM bytes per kernel family from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md § HBM)
# over tools/fwd_only.py (4 whole eager forwards and nothing else, the first a warm-up not counted, so every family's launches are whole forwards
# and per-forward bytes = per-launch bytes x launches per forward), summarised by tools/pmc_family.py into the file bench.py reads as
# profiles/rNN/pmc_families.json.   usage: tools/pmc_bench.sh <tag> <dominant family>
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; fam=$2
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "gpurun_out/pmc_${tag}_$c"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -f csv -d "gpurun_out/pmc_${tag}_$c" -o p -- \
    python3 tools/fwd_only.py 4 > /dev/null
done
python3 tools/pmc_family.py "$(find gpurun_out/pmc_${tag}_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
  "$(find gpurun_out/pmc_${tag}_WRITE_SIZE -name '*counter_collection.csv' | head -1)" "$fam" \
  "gpurun_out/pmc_families_${tag}.json" > /dev/null
echo "pmc $tag done"
