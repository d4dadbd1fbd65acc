#!/bin/bash
# gpurun with waits for an available box: retries only while gpurun reports that no box could be
# had (nothing ran, nothing charged); any run that started is final.  usage: tools/gr.sh TIMEOUT 'cmd'
t=$1; shift
for i in 1 2 3 4 5 6 7 8 9 10; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then exit $rc; fi
  echo "[gr] no box (attempt $i), waiting 60 s"; sleep 60
done
exit $rc
