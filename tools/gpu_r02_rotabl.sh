# Rotated fold ablations (fold probe only; diagnostic builds under build/).
mkdir -p gpurun_out
for lib in default build/libpacmann_abl1.so build/libpacmann_abl2.so build/libpacmann_hpl7.so build/libpacmann_hpl4.so; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_fold || exit 1
done
PM_FOLD_ROT=0 timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_fold
