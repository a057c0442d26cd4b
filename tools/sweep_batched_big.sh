#!/bin/bash
# batched serving at larger session counts (tools/batched_probe.py, 46 queries = 2 maintenance windows)
# usage: tools/sweep_batched_big.sh ["--sessions S --groups G --threads T" ...]
mkdir -p gpurun_out
if [ $# -eq 0 ]; then set -- "--sessions 256 --groups 4 --threads 16" "--sessions 384 --groups 4 --threads 16" "--sessions 512 --groups 4 --threads 16"; fi
for a in "$@"; do
  timeout -k 10 250 python -u tools/batched_probe.py --queries 46 $a >> gpurun_out/ab.log 2>&1 || exit 1
done
