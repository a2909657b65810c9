#!/bin/bash
# round-2 call 24: fused stacks phase isolation, part 2: no A loads (16), no epilogue (32), only B reads + skeleton (52)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
L=$PWD/textmae-image-compression_amd/lib
bash tools/gpu_session.sh \
  "lstk:200:python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_w0:200:TMAE_LSTK_FLAGS=0 python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d16:200:TMAE_LIB=$L/libtmae_d16.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d32:200:TMAE_LIB=$L/libtmae_d32.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms" \
  "lstk_d52:200:TMAE_LIB=$L/libtmae_d52.so python -u tools/lstk_bench.py ms_3 lrp_3 b_ms"
