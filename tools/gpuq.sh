#!/bin/bash
# Queue a gpurun call: re-submits only while the pool reports no free slot / box (the call did not run,
# nothing charged); any call that ran — passed or failed — ends the loop. usage: tools/gpuq.sh TIMEOUT 'CMD'
T=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$1" > /tmp/gpuq.out 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json'))['status'])" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then tail -3 /tmp/gpuq.out; exit $rc; fi
  sleep 60
done
echo "gave up waiting for a slot"; exit 3
