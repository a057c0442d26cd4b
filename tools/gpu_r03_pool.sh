#!/bin/bash
# Round 3: pooled batched serving: parity (batched sessions, full-size SIFT1M sessions), then the
# SIFT1M block of the bench with the pool (default) and the per-team workers (PM_BATCH_POOL=0).
out=gpurun_out/r03pool
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -k "sessions_batched or sift1m_full_sessions" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/sweep_bench.sh $out/pool "--groups 4" "--groups 6" "--groups 8" || exit 1
PM_BATCH_POOL=0 bash tools/sweep_bench.sh $out/team "--groups 4" "--groups 6" || exit 1
bash tools/sweep_bench.sh $out/pool2 "--groups 4" "--groups 6" || exit 1
