#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
G="python -u tools/gemm_bench.py enc_qkv enc_fc1 enc_fc2 enc_proj dec_qkv dec_fc1 dec_fc2 dec_proj"
bash tools/gpu_session.sh \
  "pytest_pp:300:python -u -m pytest tests/test_gpu_kernels.py -q -k 'pingpong or linear' --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "pytest_conv3:300:TMAE_CONV_TPS=3 python -u -m pytest tests/test_gpu_kernels.py -q -k conv --timeout 120 --timeout-method thread -p no:cacheprovider" \
  "conv_t1:200:TMAE_CONV_TPS=1 python -u tools/conv_bench.py" \
  "conv_t3:200:TMAE_CONV_TPS=3 python -u tools/conv_bench.py" \
  "gemm_pp0:200:TMAE_GEMM_PP=0 $G" \
  "gemm_pp1:200:TMAE_GEMM_PP=1 $G" \
  "bench_base:200:$B" \
  "bench_t3:200:TMAE_CONV_TPS=3 $B" \
  "bench_pp:200:TMAE_GEMM_PP=1 $B" \
  "bench_base2:200:$B" \
  "bench_t3b:200:TMAE_CONV_TPS=3 $B" \
  "bench_pp2:200:TMAE_GEMM_PP=1 $B"
