#!/bin/bash
# Round 3: step-kernel A/B of library builds: 64 sessions in one lock-step group alone
# (batched_probe --timing 2: per-kernel averages), builds in ABBA order.
# usage: tools/gpu_r03_mr.sh OUTDIR LIB...   ("default" = the product .so)
out=$1; shift
mkdir -p $out
libs=("$@")
rev=(); for ((i=${#libs[@]}-1; i>=0; i--)); do rev+=("${libs[$i]}"); done
for lib in "${libs[@]}" "${rev[@]}"; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  echo "$lib" >> $out/probe.log
  timeout -k 10 300 python -u tools/batched_probe.py --sessions 64 --queries 6 --timing 2 >> $out/probe.log 2>&1 || exit 1
done
