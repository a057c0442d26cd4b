#!/bin/bash
# The SIFT1M serving block at several lock-step team counts (288 sessions), ABBA.
# usage: [SWEEP="4 3 2 2 3 4"] [OUT=dir] bash tools/sweep_groups.sh
out=${OUT:-gpurun_out/sweep_g}; mkdir -p $out
B="--no-cpu-baseline --no-config2 --no-config0 --no-msmarco-search --no-bigann --no-single"
for g in ${SWEEP:-4 3 2 2 3 4}; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $B --groups $g > $out/g$g.json 2>> $out/err.log || exit 1
  python tools/ab_summary.py sift "groups=$g" $out/g$g.json | tee -a $out/summary.log
done
