#!/bin/bash
# The driver's multi-GPU bench command with 4 ranks sharing the one GPU of a
# gpurun box (round 6): configs[3] then runs as ONE 4-rank layout (shard r of
# 4 on rank r), its combine agreed over the ranks (RCCL refuses ranks that share
# a device, so the agreed fallback is gloo).  configs[4]'s 8-way shards (80 GB
# each) do not fit four to a GPU, so only configs[3] runs; the single-GPU
# blocks are skipped.
# usage: tools/rehearse4.sh OUTDIR
out=${1:-gpurun_out/rehearse4}; mkdir -p "$out"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 4 --steps 3 --warmup 1 --sessions 16 --combine rccl --big-sessions 2 \
  --bigann-blocks 3 --no-config2 --no-msmarco-search --no-single --no-config0 --no-cpu-baseline \
  > "$out/bench.json" 2> "$out/bench.err"
rc=$?; tail -c 600 "$out/bench.json"; tail -4 "$out/bench.err"; exit $rc
