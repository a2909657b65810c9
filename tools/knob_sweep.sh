#!/bin/bash
# Same-box sweep of the GEMM / conv tuning knobs (environment, no rebuild) around the default forward, plus
# forced-tile runs of the token GEMMs.   usage: tools/knob_sweep.sh (inside one gpurun call)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python bench.py --no-cpu-baseline --no-k64 --no-train --no-roofline"
tools/gpu_session.sh \
 "tiles:400:GEMM_TILES=auto,0,1,6,7,9 python tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 enc_proj dec_qkv dec_fc1 dec_fc2 dec_proj" \
 "k_base:120:$B" \
 "k_halo128:120:TMAE_CONV_HALO_BN=128 $B" \
 "k_e160lo:120:TMAE_GEMM_E160=110 $B" \
 "k_e160hi:120:TMAE_GEMM_E160=135 $B" \
 "k_e192mlo:120:TMAE_GEMM_E192M=112 $B" \
 "k_e192mhi:120:TMAE_GEMM_E192M=140 $B" \
 "k_e256lo:120:TMAE_GEMM_E256=100 $B" \
 "k_e256hi:120:TMAE_GEMM_E256=125 $B" \
 "k_base2:120:$B"
