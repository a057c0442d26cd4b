#!/bin/bash
# The default line's SIFT1M block only (no other blocks, no CPU baseline) over serving settings.
# usage: tools/sweep_bench.sh OUTDIR "ARGS1" "ARGS2" ...
out=$1; shift
mkdir -p $out
for a in "$@"; do
  echo "== $a" >> $out/sweep.log
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-single --no-bigann \
    --no-config0 --no-msmarco-search $a > $out/b.json 2>> $out/sweep.err || exit 1
  python -c "import json,sys; d=json.load(open('$out/b.json')); print(json.dumps({'args': '$a', 'qps': d['value'], 'ms_step': d['ms_per_step'], 'kernel_ms': d.get('kernel_ms')}))" >> $out/sweep.log
done
cat $out/sweep.log
