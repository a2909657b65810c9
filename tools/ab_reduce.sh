set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-base new base new}; do
  if [ $v = new ]; then unset TMAE_LIB; else export TMAE_LIB=ab/$v.so; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-k64 --no-roofline --steps 20 --warmup 5 > gpurun_out/abr_$v.log 2>&1
  grep '^{' gpurun_out/abr_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d.get('train',{}).get('value'))"
done
export TMAE_LIB=ab/base.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abr_pbase -o t -- python3 bench.py --no-cpu-baseline --no-k64 --no-roofline --steps 3 --warmup 1 > /dev/null 2>&1
unset TMAE_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/abr_pnew -o t -- python3 bench.py --no-cpu-baseline --no-k64 --no-roofline --steps 3 --warmup 1 > /dev/null 2>&1
rm -f gpurun_out/abr_p*/t_kernel_trace.csv
