# Fold slice-group width per XCD (PM_ROT_LW 1 / 2 / 4 default / 5): the serving bench's 64-client
# fold averages, each variant twice in mirrored order.
set -o pipefail
mkdir -p gpurun_out
F="--steps 40 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for v in lw1 lw2 head lw5 lw5 head lw2 lw1; do
  if [ $v = head ]; then L=""; else L="PM_LIB=$PWD/build/libpacmann_$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/lw_$v.json 2>/dev/null || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/lw_$v.json')); k=d['kernel_avg_us']; n=d['roofline_prep']
print('$v', d['value'], 'fold', k['prep_fold'], 'launches', n['launches'], 'iso fold1', d['isolated']['kernel_avg_us']['prep_fold_one_client'])"
done
