#!/bin/bash
out=gpurun_out/r03fold2
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_parity.py -k "preprocessing or batch_pir_basic or group" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for lib in default build/libpacmann_ord0.so build/libpacmann_ord0.so default; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/group_fold_probe.py 64 4 >> $out/probe.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/fold_probe.py >> $out/probe.log 2>&1 || exit 1
done
grep prep_fold $out/probe.log
