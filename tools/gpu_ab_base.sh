# Same-box A/B of the serving bench: the round-start library (build/libpacmann_base.so) vs the tree's.
mkdir -p gpurun_out
F="--steps 60 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-msmarco-search"
for i in 1 2 3; do
  PM_LIB=$PWD/build/libpacmann_base.so timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_base$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py $F > gpurun_out/ab_head$i.json 2>/dev/null || exit 1
  python -c "
import json
for n in ['ab_base$i','ab_head$i']:
    d=json.load(open(f'gpurun_out/{n}.json')); print(n, d['value'], d['single_session']['queries_per_s'], sum(v for v in d['kernel_ms'].values()))"
done
