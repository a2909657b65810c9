#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OLD=TMAE_LIB=$PWD/textmae-image-compression_amd/lib/libtmae_old.so
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_conv:300:python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "conv_new:200:python -u tools/conv_bench.py" \
  "conv_old:200:$OLD python -u tools/conv_bench.py" \
  "bench_new:200:$B" \
  "bench_old:200:$OLD $B" \
  "bench_new2:200:$B" \
  "bench_old2:200:$OLD $B"
