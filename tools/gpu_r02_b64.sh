mkdir -p gpurun_out
PM_LIB=$PWD/build/libpacmann_b64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "preprocessing or batch_pir_sequence" > gpurun_out/t_b64.log 2>&1 || { echo PARITY_FAIL; tail -20 gpurun_out/t_b64.log; exit 1; }
tail -1 gpurun_out/t_b64.log
for i in 1 2; do
for lib in default build/libpacmann_b64.so; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 120 python -u tools/fold_probe.py 2>&1 | grep prep_fold || exit 1
done
done
