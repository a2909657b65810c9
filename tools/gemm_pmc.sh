#!/bin/bash
# SQ stall breakdown of the token GEMMs beside hipBLASLt's on the same shapes: one rocprofv3 --pmc pass (8 SQ
# counters + the GRBM clock) over eager launches of tools/gemm_bench.py, summarised per kernel by tools/sq_summary.py.
#   usage: tools/gemm_pmc.sh <tag> [shape ...]      (on the GPU box; output gpurun_out/gemm_pmc_<tag>.txt)
set -e
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/gpmc_$tag
rm -rf "$out"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d "$out" -o p -- \
  python3 tools/gemm_bench.py --eager 4 "$@" > "gpurun_out/gemm_pmc_${tag}.log" 2>&1
python3 tools/sq_summary.py "$(find "$out" -name '*.db' | head -1)" > "gpurun_out/gemm_pmc_${tag}.txt"
rm -rf "$out"
