#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_relayout:300:python -u -m pytest tests/test_gpu_train.py -q -k relayout --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "train_wall:300:python -u tools/train_only.py 5" \
  "conv_bench:300:python -u tools/conv_bench.py" \
  "gemm_bench:300:python -u tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 enc_proj dec_qkv dec_fc1 dec_fc2 dec_proj" \
  "fwd_trace:300:rocprofv3 --kernel-trace -d gpurun_out/fprof -o f -f csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline --no-train"
