#!/bin/bash
# round-2 call 43: dh=32 attention at 7 waves per SIMD (3 workgroups per CU) vs 5 -- A/B of two builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
W7=textmae-image-compression_amd/lib/libtmae_w7.so
bash tools/gpu_session.sh \
  "tests_attn:300:TMAE_LIB=$W7 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k mha" \
  "bench_base:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_w7:400:TMAE_LIB=$W7 python -u bench.py --no-train --no-cpu-baseline" \
  "bench_base2:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_w7b:400:TMAE_LIB=$W7 python -u bench.py --no-train --no-cpu-baseline"
