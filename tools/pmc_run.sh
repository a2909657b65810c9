#!/bin/bash
# two PMC passes (kernel trace + one TCC counter each) over the roofline kernel, then the summary
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o f -- python3 tools/roofline_kernel.py 20
timeout -k 10 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o w -- python3 tools/roofline_kernel.py 20
python3 tools/pmc_traffic.py "$(find gpurun_out/pmc_fetch -name '*counter_collection.csv' | head -1)" \
  "$(find gpurun_out/pmc_write -name '*counter_collection.csv' | head -1)" gpurun_out/pmc_fc1_gemm.json
