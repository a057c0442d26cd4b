#!/bin/bash
# tools/rehearse4.sh with configs[0] on: the multi-rank section as the
# driver's 4-GPU run takes it (configs[0] sharded by rows, then configs[3] as
# one 4-rank layout), 4 ranks sharing one GPU (gloo fallbacks: RCCL refuses a
# shared device).
# usage: tools/rehearse4_ip.sh OUTDIR
out=${1:-gpurun_out/rehearse4_ip}; mkdir -p "$out"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29536 bench.py --gpus 4 --steps 3 --warmup 1 --sessions 16 --combine rccl --big-sessions 2 \
  --bigann-blocks 3 --no-config2 --no-msmarco-search --no-single --no-cpu-baseline \
  > "$out/bench.json" 2> "$out/bench.err"
rc=$?; tail -c 600 "$out/bench.json"; tail -4 "$out/bench.err"; exit $rc
