#!/bin/bash
# round-2 call 2: DP/optimizer tests, bench, HBM traffic of the dominant family, attention PMC
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python3 bench.py --no-graph --steps 2 --warmup 1 --no-train --no-cpu-baseline --no-roofline"
bash tools/gpu_session.sh \
  "pytest_dp:400:python -u -m pytest tests/test_gpu_optim_dp.py -v --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "bench:400:python -u bench.py > gpurun_out/bench.json" \
  "pmc_fetch:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc FETCH_SIZE -f csv -d gpurun_out/pmc_fetch -o f -- $B" \
  "pmc_write:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc WRITE_SIZE -f csv -d gpurun_out/pmc_write -o w -- $B" \
  "attn_bench:120:python -u tools/attn_bench.py" \
  "attn_pmc1:90:timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE -f csv -d gpurun_out/attn_pmc1 -o a -- python3 tools/attn_only.py dec 5" \
  "attn_pmc2:90:timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU -f csv -d gpurun_out/attn_pmc2 -o a -- python3 tools/attn_only.py dec 5"
