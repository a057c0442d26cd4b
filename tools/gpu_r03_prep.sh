#!/bin/bash
out=gpurun_out/r03prep
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -k "sessions_batched or sift1m_full_sessions" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-single --no-bigann --no-config0 --no-msmarco-search"
for i in 1 2; do
  for cfg in "PM_PREP_WAIT_MS=0" "PM_PREP_WAIT_MS=10" "PM_PREP_WAIT_MS=30"; do
    env $cfg timeout -k 10 200 python -u bench.py $B > $out/b.json 2>> $out/err.log || exit 1
    python -c "import json; d=json.load(open('$out/b.json')); print('$cfg', d['value'], d['ms_per_step'], d['maintenance_s_per_query'], d['kernel_avg_us'].get('prep_fold'))" | tee -a $out/summary.log
  done
done
