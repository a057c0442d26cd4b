#!/bin/bash
out=gpurun_out/r03gather
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_shard_search_gpu.py -k "bigann or synth or 1b or shard" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-single --no-config0 --no-msmarco-search"
for lib in default build/libpacmann_gold.so build/libpacmann_gold.so default; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u bench.py $B > $out/b.json 2>> $out/err.log || exit 1
  python -c "
import json; d=json.load(open('$out/b.json'))
for c in ('config3_bigann_100m','config4_bigann_1b'):
    x=d[c]; print('$lib', c, x['private_queries_per_s'], x['ms_per_round'], x['kernel_avg_us'].get('gather'), x['kernel_avg_us'].get('answer'))" | tee -a $out/summary.log
done
