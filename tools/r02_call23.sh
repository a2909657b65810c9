#!/bin/bash
# round-2 call 23: fused stacks: zero block for border taps; phase isolation (no MFMA / no B reads / no A loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=$PWD/textmae-image-compression_amd/lib
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"
bash tools/gpu_session.sh \
  "pytest_lstk:300:python -u -m pytest tests/test_gpu_lic_stack.py -q --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "lstk:200:python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d4:200:TMAE_LIB=$L/libtmae_d4.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d8:200:TMAE_LIB=$L/libtmae_d8.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "pmc2:90:timeout -s KILL 80 rocprofv3 --kernel-trace --pmc $P2 -f csv -d gpurun_out/pmc2 -o p -- python3 tools/lstk_bench.py ms_3"
