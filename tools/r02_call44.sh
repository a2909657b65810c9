#!/bin/bash
# round-2 call 44: lic_stack GELU epilogue with permlane16_swap 16-B stores vs 8-B stores (libtmae_o1.so,
# -DLSTK_OPT=1): stack tests, stack micro-bench and bench A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O1=textmae-image-compression_amd/lib/libtmae_o1.so
bash tools/gpu_session.sh \
  "tests_lstk:300:python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_lic_stack.py tests/test_gpu_mcm.py" \
  "lstk_new:200:python -u tools/lstk_bench.py" \
  "lstk_o1:200:TMAE_LIB=$O1 python -u tools/lstk_bench.py" \
  "bench_new:400:python -u bench.py --no-train --no-cpu-baseline" \
  "bench_o1:400:TMAE_LIB=$O1 python -u bench.py --no-train --no-cpu-baseline" \
  "bench_new2:400:python -u bench.py --no-train --no-cpu-baseline"
