#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_mha:300:python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_train.py -q -k 'mha' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "attn_bench:200:python -u tools/attn_bench.py" \
  "conv_d0:200:TMAE_CONV_DIAG=0 python -u tools/conv_bench.py" \
  "conv_d1:200:TMAE_CONV_DIAG=1 python -u tools/conv_bench.py" \
  "conv_d2:200:TMAE_CONV_DIAG=2 python -u tools/conv_bench.py" \
  "conv_d4:200:TMAE_CONV_DIAG=4 python -u tools/conv_bench.py" \
  "conv_d8:200:TMAE_CONV_DIAG=8 python -u tools/conv_bench.py" \
  "conv_d6:200:TMAE_CONV_DIAG=6 python -u tools/conv_bench.py" \
  "conv_d10:200:TMAE_CONV_DIAG=10 python -u tools/conv_bench.py" \
  "conv_d14:200:TMAE_CONV_DIAG=14 python -u tools/conv_bench.py" \
  "conv_d15:200:TMAE_CONV_DIAG=15 python -u tools/conv_bench.py"
