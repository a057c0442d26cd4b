#!/bin/bash
# Group-fold A/B: the 64-client group-preprocessing parity test on the product
# build, then tools/group_fold_probe.py on each build, twice in ABBA order.
# usage: tools/gpu_fold_ab.sh OUTDIR LIB...   ("default" = the product .so)
out=$1; shift
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 500 --timeout-method thread \
  -k group_preprocessing > "$out/test.log" 2>&1 || { tail -5 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
libs=("$@")
rev=(); for ((i=${#libs[@]}-1; i>=0; i--)); do rev+=("${libs[$i]}"); done
for lib in "${libs[@]}" "${rev[@]}"; do
  if [ "$lib" = default ]; then unset PM_LIB; else export PM_LIB=$PWD/$lib; fi
  timeout -k 10 300 python -u tools/group_fold_probe.py 64 4 >> "$out/probe.log" 2>&1 || { tail -5 "$out/probe.log"; exit 1; }
done
cat "$out/probe.log"
