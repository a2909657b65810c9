#!/bin/bash
# round-2 call 22: fused stacks v5 (LDS tap masks): tests, micro-bench policy A vs B, PMC, forward A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
bash tools/gpu_session.sh \
  "pytest_lstk:300:python -u -m pytest tests/test_gpu_lic_stack.py -v -s --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "lstkA:200:TMAE_LSTK_FLAGS=1 python -u tools/lstk_bench.py" \
  "lstkB:200:TMAE_LSTK_FLAGS=3 python -u tools/lstk_bench.py" \
  "pmc1:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $P1 -f csv -d gpurun_out/pmc1 -o p -- python3 tools/lstk_bench.py ms_3" \
  "pmc2:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $P2 -f csv -d gpurun_out/pmc2 -o p -- python3 tools/lstk_bench.py ms_3" \
  "bench_A:200:TMAE_LSTK_FLAGS=1 $B" \
  "bench_B:200:TMAE_LSTK_FLAGS=3 $B" \
  "bench_old:200:TMAE_LIC_STACK=0 $B"
