#!/bin/bash
# Token-GEMM A/B of variant libraries in one GPU call: tools/gemm_bench.py under each TMAE_LIB (the in-tree library
# is "base"), interleaved twice so box drift shows.   usage: tools/gemm_ab.sh <tag> <variant> ... [-- shape ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
vars=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
[ "$1" = "--" ] && shift
mkdir -p gpurun_out
for rep in 1 2; do
  for v in base "${vars[@]}"; do
    if [ "$v" = base ]; then lib=""; else lib="ab/libtmae_$v.so"; fi
    echo "=== $v rep $rep" >> "gpurun_out/gab_$tag.log"
    TMAE_LIB=$lib timeout -k 10 240 python tools/gemm_bench.py "$@" 2>&1 | tail -1 >> "gpurun_out/gab_$tag.log" || exit $?
  done
done
echo done
