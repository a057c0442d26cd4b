# Two-rank rehearsal of the driver's multi-GPU bench command on one GPU (ranks share cuda:0;
# the BIGANN combine over gloo, since RCCL refuses two ranks on one device).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 3 --combine gloo > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -30 gpurun_out/rehearse2.err; exit 1; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/rehearse2.json"))
print(d["value"], d["n_gpus"], d["config"].get("parallelism"), d.get("scaling"))
for k in ("config3_bigann_100m", "config4_bigann_1b"):
    b = d.get(k, {})
    print(k, b.get("error") or {x: b.get(x) for x in ("n_ranks", "combine", "private_queries_per_s", "mismatches", "ms_per_round")})
PY
