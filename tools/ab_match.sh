#!/bin/bash
# A/B of the two k_match forms in batched serving (PM_MATCH_PART=0: per sub-query; -1: auto).
mkdir -p gpurun_out
for v in 0 -1 0 -1; do
  PM_MATCH_PART=$v timeout -k 10 200 python -u tools/batched_probe.py --sessions 128 --groups 4 --threads 8 --queries 15 --timing 2 >> gpurun_out/bp.log 2>&1 || exit 1
  echo "variant $v" >> gpurun_out/bp.log
done
