# same-box A/B of an environment knob on the bench (forward + training lines): usage ENVSET="K=V" bash tools/ab_env.sh
set -e
mkdir -p gpurun_out
for v in base knob base knob; do
  if [ $v = knob ]; then export $ENVSET; else unset ${ENVSET%%=*}; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-k64 --no-roofline --steps 20 --warmup 5 > gpurun_out/abe_$v.log 2>&1
  grep '^{' gpurun_out/abe_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d.get('train',{}).get('value'))"
done
