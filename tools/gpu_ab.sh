# A/B of the SIFT1M serving bench on one box: trees under build/<name>tree vs this tree, alternating
set -o pipefail
F="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for i in 1 2; do
  for t in "$@"; do
    if [ "$t" = cur ]; then timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_$t$i.json 2>/dev/null || exit 1
    else (cd build/${t}tree && timeout -k 10 300 python -u bench.py $F > ../../gpurun_out/ab_$t$i.json 2>/dev/null) || exit 1; fi
    python -c "
import json; d=json.load(open('gpurun_out/ab_$t$i.json')); k=d['kernel_avg_us']; iso=(d.get('isolated') or {}).get('kernel_avg_us', {})
print('$t$i', d['value'], {x: k.get(x) for x in ('hint_match','resolve','answer','prep_fold','prep_offsets')}, iso)"
  done
done
