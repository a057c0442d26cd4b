# A/B of the SIFT1M serving bench: round-1 tree (build/r01tree) vs this tree, alternating on one box
set -o pipefail
F="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single"
for i in 1 2; do
  (cd build/r01tree && timeout -k 10 300 python -u bench.py $F > ../../gpurun_out/ab_old$i.json 2>/dev/null) || exit 1
  timeout -k 10 300 python -u bench.py $F --no-msmarco-search --no-kernel-timing > gpurun_out/ab_new$i.json 2>/dev/null || exit 1
  PM_ROWS_CHECK=0 timeout -k 10 300 python -u bench.py $F --no-msmarco-search --no-kernel-timing > gpurun_out/ab_nochk$i.json 2>/dev/null || exit 1
  python -c "import json;print('old', json.load(open('gpurun_out/ab_old$i.json'))['value'], 'new', json.load(open('gpurun_out/ab_new$i.json'))['value'], 'nocheck', json.load(open('gpurun_out/ab_nochk$i.json'))['value'])"
done
