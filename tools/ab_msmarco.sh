#!/bin/bash
# Same-box ABBA of library builds on the MS-MARCO private-search block (64 sessions, 2 teams).
# usage: bash tools/ab_msmarco.sh OUTDIR default|path/to/lib.so ...
out=$1; shift
vars=("$@"); rev=(); for ((i=${#vars[@]}-1; i>=0; i--)); do rev+=("${vars[$i]}"); done
n=0
for v in "${vars[@]}" "${rev[@]}"; do
  n=$((n+1))
  if [ "$v" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$v; fi
  echo "== run$n $v"
  bash tools/sweep_msmarco.sh "$out/run$n" 64:2 || exit 1
done
exit 0
