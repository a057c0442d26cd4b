#!/bin/bash
# A/B diagnostic builds: tools/ab_libs.sh var/libA.so var/libB.so ...  ("default" = the product .so)
# each: preprocessing parity subset, then tools/fold_probe.py twice -> gpurun_out/fold_ab.log
mkdir -p gpurun_out
for lib in "$@"; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "prf or preprocessing or batch_pir or bigann_partition or group" > gpurun_out/t_$(basename $lib).log 2>&1 \
    || { echo "PARITY FAIL $lib"; exit 1; }
done
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
    timeout -k 10 120 python -u tools/fold_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit 1
  done
done
echo done
