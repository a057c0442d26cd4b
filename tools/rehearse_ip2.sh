#!/bin/bash
# configs[0] sharded by rows over 2 ranks sharing the one GPU of a gpurun box
# (round 6): each rank scans half of the 1e8-row fill, the two mod-2^32 sums
# meet in one all-reduce (the agreed RCCL group, else gloo: RCCL refuses two
# ranks on one device), the total is checked against the closed form.
# usage: tools/rehearse_ip2.sh OUTDIR
out=${1:-gpurun_out/rehearse_ip2}; mkdir -p "$out"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29535 bench.py --gpus 2 --steps 3 --warmup 1 --sessions 16 --no-bigann --no-config2 \
  --no-msmarco-search --no-single --no-cpu-baseline > "$out/bench.json" 2> "$out/bench.err"
rc=$?; tail -c 600 "$out/bench.json"; tail -4 "$out/bench.err"; exit $rc
