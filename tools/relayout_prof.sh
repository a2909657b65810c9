mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in nt t conv conv_dg; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/rlk_$k -o t -- python3 tools/relayout_bench.py $k > /dev/null 2>&1 || exit 1
  rm -f gpurun_out/rlk_$k/t_kernel_trace.csv
done
