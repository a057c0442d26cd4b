#!/bin/bash
# A/B of an environment switch on batched serving: tools/ab_env.sh VAR "v1 v2 v1 v2" [probe args...]
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
for v in $vals; do
  env $var=$v timeout -k 10 200 python -u tools/batched_probe.py "$@" >> gpurun_out/ab.log 2>&1 || exit 1
  echo "$var=$v" >> gpurun_out/ab.log
done
