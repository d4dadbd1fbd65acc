#!/bin/bash
# Development: submit one gpurun call, resubmitting it only while the pool answers "no box / slot
# free" (exit 3: nothing ran, nothing charged).  Any other outcome, pass or fail, ends the loop.
#   tools/gpurun_wait.sh <out-file> <gpurun timeout s> '<command>'
out=$1; lim=$2; cmd=$3
for i in $(seq 1 30); do
  timeout $((lim + 1500)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
