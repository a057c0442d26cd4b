# Rotated fold ablations, one-client SIFT1M preprocessing (tools/fold_probe.py):
# default, PM_ROT_ABL=1 (no LDS reads), PM_ROT_ABL=2 (no staging in the loop).
mkdir -p gpurun_out
for i in 1 2; do
for lib in default build/libpacmann_abl1.so build/libpacmann_abl2.so "$@"; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_ || exit 1
done
done
