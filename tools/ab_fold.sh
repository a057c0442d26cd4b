#!/bin/bash
# preprocessing parity + kernel timing (SIFT1M shape): tools/ab_fold.sh TAG
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "prf or preprocessing or batch_pir_sequence or bigann_partition" > gpurun_out/t_fold.log 2>&1 || exit 1
for i in 1 2; do timeout -k 10 120 python -u tools/fold_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit 1; done
echo "$1" >> gpurun_out/fold_ab.log
