#!/bin/bash
# round-2 call 31: halo conv with two images per workgroup (TMAE_CONV_HALO_IMG=2): bitwise test, conv micro-bench,
# forward A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "pytest_conv:300:python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "conv1:200:TMAE_CONV_HALO_IMG=1 python -u tools/conv_bench.py ha_384_384 first_96_224" \
  "conv2:200:TMAE_CONV_HALO_IMG=2 python -u tools/conv_bench.py ha_384_384 first_96_224" \
  "bench_i1:200:TMAE_CONV_HALO_IMG=1 $B" \
  "bench_i2:200:TMAE_CONV_HALO_IMG=2 $B" \
  "bench_i1b:200:TMAE_CONV_HALO_IMG=1 $B" \
  "bench_i2b:200:TMAE_CONV_HALO_IMG=2 $B"
