#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_session.sh \
  "pytest_vgg_attn:600:python -u -m pytest tests/test_gpu_vgg.py tests/test_gpu_kernels.py tests/test_gpu_train.py -q -k 'vgg or mha or attn or feature or maxpool' --timeout 240 --timeout-method thread -p no:cacheprovider" \
  "attn_per1:120:TMAE_MHA_PER=1 python -u tools/attn_bench.py" \
  "attn_auto:120:python -u tools/attn_bench.py" \
  "attn_per3:120:TMAE_MHA_PER=3 python -u tools/attn_bench.py" \
  "attn_per4:120:TMAE_MHA_PER=4 python -u tools/attn_bench.py" \
  "bench:400:python -u bench.py --no-train --no-cpu-baseline > gpurun_out/bench.json"
