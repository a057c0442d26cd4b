# k_answer variants: phase stamps of one lock-step group alone, then the contended bench value
set -o pipefail
F="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for v in w6k12 w8k8 w8k12; do
  rm -f gpurun_out/st_$v.bin
  PM_LIB=build/libpacmann_st_$v.so PM_ANSWER_STAMPS=gpurun_out/st_$v.bin timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search --sessions 64 --groups 1 > /dev/null 2>&1 || exit 1
  echo "== $v isolated"; python tools/answer_stamps.py gpurun_out/st_$v.bin; rm -f gpurun_out/st_$v.bin
done
for i in 1 2; do
  for v in w6k12 w8k8 w8k12; do
    L=build/libpacmann_$v.so; [ $v = w6k12 ] && L=pacmann_amd/libpacmann.so
    PM_LIB=$L timeout -k 10 300 python -u bench.py $F > gpurun_out/var_$v$i.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/var_$v$i.json')); k=d['kernel_avg_us']
print('$v$i', d['value'], 'answer', k['answer'], 'iso', d['isolated']['kernel_avg_us']['answer'], 'match', k['hint_match'])"
  done
done
