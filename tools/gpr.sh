#!/bin/bash
# gpurun with retries on infrastructure-side transients only (nothing ran, nothing charged).
# usage: tools/gpr.sh TIMEOUT 'command'
t=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
  echo "$out" | tail -n 6
  # retry only when the call's own status line says nothing ran (a finished
  # call's tail can quote such words from earlier attempts)
  if echo "$out" | grep -q "^\[gpurun\] status=transient" && ! echo "$out" | grep -q "^\[gpurun\] status=ok"; then sleep 90; continue; fi
  if [ $rc -eq 3 ] || { ! echo "$out" | grep -q "^\[gpurun\] status=" && echo "$out" | grep -q "no free box\|slot(s) on this pod are busy"; }; then sleep 90; continue; fi
  exit $rc
done
exit $rc
