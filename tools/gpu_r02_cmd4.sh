set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests4.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|error" gpurun_out/gputests4.log | head -20; tail -5 gpurun_out/gputests4.log; exit 1; }
tail -2 gpurun_out/gputests4.log
F="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $F > gpurun_out/c4_new$i.json 2>/dev/null || exit 1
  PM_LIB=build/libpacmann_pub4.so timeout -k 10 300 python -u bench.py $F > gpurun_out/c4_pub4_$i.json 2>/dev/null || exit 1
  python -c "
import json
for n in ['c4_new$i','c4_pub4_$i']:
    d=json.load(open(f'gpurun_out/{n}.json')); print(n, d['value'], d['kernel_avg_us'], d['isolated']['kernel_avg_us'])"
done
