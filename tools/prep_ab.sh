#!/bin/bash
# group preprocessing time (kernel averages) with maintenance inside the window
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/batched_probe.py --sessions 128 --groups 4 --threads 8 --queries 40 --timing 1 >> gpurun_out/prep_ab.log 2>&1
