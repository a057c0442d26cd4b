#!/bin/bash
# Same-box ABBA of environment switches on the MS-MARCO private-search block at
# its bench shape (128 sessions, 4 teams); one line per run.
# usage: bash tools/ab_msmarco_env.sh OUTDIR default|VAR=value[,VAR=value] ...
out=$1; shift; mkdir -p "$out"
vars=("$@"); rev=(); for ((i=${#vars[@]}-1; i>=0; i--)); do rev+=("${vars[$i]}"); done
n=0
for v in "${vars[@]}" "${rev[@]}"; do
  n=$((n+1)); envs=()
  [ "$v" = default ] || IFS=, read -ra envs <<< "$v"
  f="$out/run$n"
  env "${envs[@]}" timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --sessions 8 --no-cpu-baseline \
    --no-config2 --no-config0 --no-bigann --no-single --no-kernel-timing > "$f.json" 2> "$f.err" || exit 1
  python3 -c "import json; d=json.load(open('$f.json'))['config2_private_search']; print('$v', d['private_queries_per_s'], d['online_s_per_query'], d['maintenance_s_per_query'], d['kernel_avg_us'])" | tee -a "$out/summary.log" || exit 1
done
