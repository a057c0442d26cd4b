# Serving-shape sweep of the bench's SIFT1M block (sessions / lock-step groups / workers), one box.
mkdir -p gpurun_out
F="--steps 46 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-msmarco-search --no-single --no-kernel-timing"
for a in "--sessions 256 --groups 4" "--sessions 384 --groups 4" "--sessions 512 --groups 4" "--sessions 384 --groups 6" "--sessions 512 --groups 8" "--sessions 256 --groups 4"; do
  timeout -k 10 300 python -u bench.py $F $a > gpurun_out/sw.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('$a', d['value'])"
done
