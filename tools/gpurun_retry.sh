#!/bin/bash
# Run one gpurun call, retrying ONLY while the pool has no free box (gpurun exit 3: nothing ran,
# nothing charged). Any other outcome (success, failure, refusal) ends the loop.
# usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box right now\|backing off\|status=transient" "$out"; then echo "rc=$rc"; exit $rc; fi
  sleep 120
done
echo "gave up (no box)"; exit 3
