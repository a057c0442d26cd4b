mkdir -p gpurun_out/r6g
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_aes_bs.py "tests/test_gpu_parity.py::test_device_loop_fault_marks_sessions_lost" "tests/test_gpu_parity.py::test_search_device_loop_vs_host_loop" > gpurun_out/r6g/tests_a.log 2>&1
rc=$?; tail -3 gpurun_out/r6g/tests_a.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
PM_RCCL_NONBLOCKING=1 PM_RCCL_DEBUG=1 NCCL_DEBUG=INFO timeout -k 10 600 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_shard_search_gpu.py tests/test_shard_gpu.py -k "rccl" > gpurun_out/r6g/tests_rccl_nb.log 2>&1
rc=$?; tail -3 gpurun_out/r6g/tests_rccl_nb.log; exit $rc
