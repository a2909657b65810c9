#!/bin/bash
# A/B of the GEMM variants on the hot-path shapes (tools/gemm_bench.py); diag 8 = s_setprio around MFMA blocks
python tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 dec_fc1 big > gpurun_out/ab_ring.log 2>&1 && \
GEMM_DIAG=8 python tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 dec_fc1 big > gpurun_out/ab_ring_prio.log 2>&1 && \
TMAE_GEMM_RING=0 python tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 dec_fc1 big > gpurun_out/ab_2st.log 2>&1 && \
TMAE_GEMM_RING=0 GEMM_DIAG=8 python tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 dec_fc1 big > gpurun_out/ab_2st_prio.log 2>&1
