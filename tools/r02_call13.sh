#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
G="python -u tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 enc_proj dec_qkv dec_fc1 dec_fc2 dec_proj"
bash tools/gpu_session.sh \
  "pytest_gpu:900:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "gemm_d0:200:GEMM_DIAG=0 $G" \
  "gemm_d1:200:GEMM_DIAG=1 $G" \
  "train_wall:300:python -u tools/train_only.py 5"
