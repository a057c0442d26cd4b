# k_answer workgroup size A/B (PM_ANSWER_NT: 0 = generic 512-thread / 33 KB
# LDS instance; 512 / 256 / 128 = the small-LDS instance); GPU tests first.
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests9.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests9.log | head; tail -5 gpurun_out/gputests9.log; exit 1; }
tail -1 gpurun_out/gputests9.log
F="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for i in 1 2; do
  for v in 0 512 256 128; do
    PM_ANSWER_NT=$v timeout -k 10 300 python -u bench.py $F > gpurun_out/nt_$v-$i.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/nt_$v-$i.json')); k=d['kernel_avg_us']
print('nt$v-$i', d['value'], 'answer', k['answer'], 'iso', d['isolated']['kernel_avg_us']['answer'], 'match', k['hint_match'], 'resolve', k['resolve'])"
  done
done
for v in 256 128; do
  rm -f gpurun_out/st_$v.bin
  PM_ANSWER_NT=$v PM_LIB=build/libpacmann_stamps.so PM_ANSWER_STAMPS=gpurun_out/st_$v.bin timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search --sessions 64 --groups 1 > /dev/null 2>&1 || exit 1
  echo "stamps nt=$v"; python tools/answer_stamps.py gpurun_out/st_$v.bin; rm -f gpurun_out/st_$v.bin
done
