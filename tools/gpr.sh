#!/bin/bash
# gpurun with retries on infrastructure-side transients only (nothing ran, nothing charged).
# usage: tools/gpr.sh TIMEOUT 'command'
t=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -n 6
  if echo "$out" | grep -q "status=transient\|backing off\|no box or slot"; then sleep 90; continue; fi
  exit $rc
done
exit $rc
