#!/bin/bash
# round-2 call 29: slice chain on a high-priority stream (TMAE_LIC_PRIO) A/B, graph and eager; parity tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-train"
bash tools/gpu_session.sh \
  "bench_p1:200:TMAE_LIC_PRIO=1 $B" \
  "bench_p0:200:TMAE_LIC_PRIO=0 $B" \
  "bench_p1b:200:TMAE_LIC_PRIO=1 $B" \
  "bench_p0b:200:TMAE_LIC_PRIO=0 $B" \
  "bench_p1e:200:TMAE_LIC_PRIO=1 $B --no-graph" \
  "bench_p0e:200:TMAE_LIC_PRIO=0 $B --no-graph" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 2 --no-train --no-cpu-baseline --no-roofline" \
  "pytest:900:python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_lic_stack.py tests/test_gpu_coding.py tests/test_gpu_mcm.py -q --timeout 300 --timeout-method thread -p no:cacheprovider"
