# Rotated fold from the DB image: preprocessing/batch parity subset, fold probe (default, ablations, old pipe).
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "preprocessing or batch_pir or group or sessions" > gpurun_out/t_rot.log 2>&1 || { echo PARITY_FAIL; tail -30 gpurun_out/t_rot.log; exit 1; }
tail -1 gpurun_out/t_rot.log
for lib in default build/libpacmann_abl1.so build/libpacmann_abl2.so; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_fold || exit 1
done
unset PM_LIB
PM_FOLD_ROT=0 timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_fold
