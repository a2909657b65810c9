#!/bin/bash
# gpurun with waiting for a free box: re-submits ONLY while gpurun answers 3 ("no box or slot free right now",
# nothing ran, nothing charged), every 120 s, at most 20 times.  Any other exit (including a failed GPU step) is
# returned as is.   usage: tools/gpurun_wait.sh <out.txt> <timeout_s> '<command>'
out=$1; tmo=$2; cmd=$3
for i in $(seq 1 20); do
  timeout $((tmo + 900)) /usr/local/graft/bin/gpurun --timeout "$tmo" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 120
done
exit 3
