#!/bin/bash
# Sessions / teams sweep of the MS-MARCO d=192 private-search block (the SIFT1M
# line runs too, value only); each run under its own time limit, stop at the first failure.
# usage: bash tools/sweep_msmarco.sh OUTDIR "S:G" ...
out=$1; shift
mkdir -p "$out"
for sg in "$@"; do
  S=${sg%%:*}; G=${sg##*:}
  f="$out/ms_s${S}_g${G}"
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 --ms-sessions $S --ms-groups $G --no-cpu-baseline \
    --no-config2 --no-config0 --no-bigann --no-single --no-kernel-timing > "$f.json" 2> "$f.err" || exit 1
  python3 -c "import json; d=json.load(open('$f.json'))['config2_private_search']; print('S=$S G=$G', d['private_queries_per_s'], d['recall_at_10'], d['online_s_per_query'], d['maintenance_s_per_query'], d['kernel_avg_us'])" || exit 1
done
exit 0
