#!/bin/bash
# Same-box ABBA A/B of two builds (PM_LIB) on the SIFT1M serving line.
# usage: tools/ab_libs_bench.sh OUTDIR LIB_A LIB_B [bench args]
out=$1; a=$2; b=$3; shift 3
mkdir -p $out
args=${*:---steps 20 --warmup 5}
i=0
for l in $a $b $b $a; do
  i=$((i+1))
  PM_LIB=$l timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-config2 --no-msmarco-search \
    --no-config0 --no-bigann > $out/run$i.json 2>> $out/err.log || exit 1
  echo "$i $l $(python3 -c "import json; d=json.load(open('$out/run$i.json')); print(d['value'], d['ms_per_step'], round(d['host_ms']['host_knn_update']), round(d['host_ms']['host_gvi_parse']))")"
done
