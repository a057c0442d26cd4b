#!/bin/bash
# k_match_part8 (one wave per hint block, 16-B search-row loads) vs the
# LDS-merged k_match_part: parity of the batched / BIGANN paths, then ABBA
# BIGANN bench lines with PM_MATCH_PART8=1 / 0.
out=gpurun_out/r03match8
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  tests/test_shard_search_gpu.py -k "bigann or synth or 1b or shard or batched or group" > $out/tests.log 2>&1
rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-single --no-config0 --no-msmarco-search"
for v in 1 0 0 1; do
  PM_MATCH_PART8=$v timeout -k 10 300 python -u bench.py $B > $out/b.json 2>> $out/err.log || exit 1
  python -c "
import json; d=json.load(open('$out/b.json'))
for c in ('config3_bigann_100m','config4_bigann_1b'):
    x=d[c]; k=x['kernel_avg_us']; print('part8=$v', c, x['private_queries_per_s'], x['ms_per_round'], k.get('hint_match'), k.get('resolve'), k.get('gather'), k.get('answer'))" | tee -a $out/summary.log
done
