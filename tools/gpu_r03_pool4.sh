#!/bin/bash
out=gpurun_out/r03pool4
mkdir -p $out
B="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-single --no-bigann --no-config0 --no-msmarco-search"
for a in "PM_BATCH_POOL=0 --groups 4" "x --groups 4" "x --groups 4 --threads 20" "x --groups 4 --threads 24" "x --groups 6" "x --groups 8" "x --groups 4" "PM_BATCH_POOL=0 --groups 4" "x --groups 6 --threads 20"; do
  env=${a%% *}; args=${a#* }
  [ "$env" = x ] && env="PM_BATCH_POOL=1"
  env $env timeout -k 10 200 python -u bench.py $B $args > $out/b.json 2>> $out/err.log || exit 1
  python -c "import json; d=json.load(open('$out/b.json')); h=d['host_ms']; n=256*400; print('$a', d['value'], d['ms_per_step'], {k: round(v/n*1e3,2) for k,v in h.items() if k in ('host_knn_update','host_batch_query','host_gvi_parse')})" | tee -a $out/summary.log
done
