mkdir -p gpurun_out/help3
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "batch_pir or search_knn or search_loop or batch_query" > gpurun_out/help3/tests.log 2>&1 || exit 1
PM_LIB=pacmann_amd/libpacmann_ststamps.so PM_STAMP_FILE=gpurun_out/help3/c2.bin timeout -k 10 300 python -u tools/step_stamps.py --run --c2 > gpurun_out/help3/run.log 2>&1 || exit 1
python tools/step_stamps.py --show gpurun_out/help3/c2.bin > gpurun_out/help3/show.txt 2>&1
for h in 0 3 4 5 5 4 3 0; do
  echo "== PM_STEP_HELP=$h" >> gpurun_out/help3/host.log
  PM_STEP_HELP=$h timeout -k 10 300 python -u tools/batchpir_host.py 200 >> gpurun_out/help3/host.log 2>&1 || exit 1
done
