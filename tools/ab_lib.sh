#!/bin/bash
# Same-box A/B of the in-tree library against ab/libtmae_old.so (built by hand from the previous source):
# bench (inference only) new, old, new; then one rocprofv3 kernel-stats pass of the new build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=textmae-image-compression_amd/lib/libtmae.so
B="python bench.py --no-train --no-cpu-baseline"
cp $L gpurun_out/new.so.bak || exit 1
tools/gpu_session.sh "pytest_gpu:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench_new:200:$B" || exit $?
cp ab/libtmae_old.so $L && tools/gpu_session.sh "bench_old:200:$B"; rc=$?
cp gpurun_out/new.so.bak $L && rm gpurun_out/new.so.bak
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}"
tools/gpu_session.sh "bench_new2:200:$B" \
  "prof:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --no-train --no-cpu-baseline --steps 20"
