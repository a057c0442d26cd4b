#!/bin/bash
# The driver's multi-GPU bench command with 2 ranks sharing the one GPU of a
# gpurun box (RCCL refuses two ranks on one device: the sharded blocks combine
# over gloo here; COMBINE=rccl exercises the agreed fallback: both ranks' RCCL
# setups fail on the shared device, and the ranks agree on gloo).
# usage: [COMBINE=rccl|gloo] tools/rehearse2.sh OUTDIR
out=${1:-gpurun_out/rehearse2}; mkdir -p "$out"
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --sessions 32 --combine ${COMBINE:-gloo} --big-sessions 2 \
  > "$out/bench.json" 2> "$out/bench.err"
rc=$?; tail -c 400 "$out/bench.json"; tail -4 "$out/bench.err"; exit $rc
