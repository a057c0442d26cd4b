#!/bin/bash
# Round 3: fold/match-resolve change set on one box: parity subset, fold A/B (SIFT1M 64 clients,
# MS-MARCO 32 clients), match_resolve stamps old vs new.
out=gpurun_out/r03fold
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_parity.py -k "prf or preprocessing or batch_pir or bigann_partition or group or search" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for lib in default build/libpacmann_old.so build/libpacmann_ord0.so build/libpacmann_g4s8.so default; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/group_fold_probe.py 64 4 >> $out/probe.log 2>&1 || exit 1
done
for lib in default build/libpacmann_old.so default; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/group_fold_probe.py 32 2 msmarco >> $out/probe.log 2>&1 || exit 1
done
unset PM_LIB
grep prep_fold $out/probe.log
for v in mrst_old mrst; do
  PM_LIB=$PWD/build/libpacmann_$v.so PM_MR_STAMPS=$PWD/$out/st_$v.bin timeout -k 10 300 python -u tools/batched_probe.py --sessions 64 --queries 4 --timing 1 > $out/mr_$v.log 2>&1 || exit 1
  python tools/mr_stamps.py $out/st_$v.bin
done
