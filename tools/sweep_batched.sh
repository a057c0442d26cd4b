#!/bin/bash
# Throughput sweep of batched serving (tools/batched_probe.py) over sessions / groups / threads.
mkdir -p gpurun_out
q=${Q:-15}
for a in "--sessions 128 --groups 4 --threads 8" "--sessions 128 --groups 4 --threads 12" "--sessions 192 --groups 4 --threads 12" "--sessions 256 --groups 4 --threads 16"; do
  timeout -k 10 250 python -u tools/batched_probe.py --queries $q $a >> gpurun_out/ab.log 2>&1 || exit 1
done
