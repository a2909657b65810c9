#!/bin/bash
# round-2 call 26: fused stacks phase isolation after the batched epilogue: no A loads (16), no A + no MFMA (20),
# no A + no epilogue (48), no L2 warm-up (flags 0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=$PWD/textmae-image-compression_amd/lib
bash tools/gpu_session.sh \
  "lstk:200:python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_w0:200:TMAE_LSTK_FLAGS=0 python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d16:200:TMAE_LIB=$L/libtmae_d16.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d20:200:TMAE_LIB=$L/libtmae_d20.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d48:200:TMAE_LIB=$L/libtmae_d48.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms"
