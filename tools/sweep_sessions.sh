#!/bin/bash
# Sessions / teams sweep of the SIFT1M line (value only: no kernel-timing pass,
# no other blocks); each run under its own time limit, stop at the first crash.
# usage: [ARGS="--stagger-teams"] [TAG=_x] bash tools/sweep_sessions.sh OUTDIR "S:G" ...
out=$1; shift
mkdir -p "$out"
for sg in "$@"; do
  S=${sg%%:*}; G=${sg##*:}
  f="$out/s${S}_g${G}${TAG}"
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --sessions $S --groups $G --no-cpu-baseline --no-config2 \
    --no-msmarco-search --no-config0 --no-bigann --no-single --no-kernel-timing $ARGS > "$f.json" 2> "$f.err"
  rc=$?
  python3 -c "import json; d=json.load(open('$f.json')); print('S=$S G=$G $ARGS', d['value'], d['ms_per_step'], d['maintenance_in_region'])" || exit 1
  [ $rc -ne 0 ] && exit $rc
done
exit 0
