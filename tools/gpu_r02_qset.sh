# Pre-expanded query sets (PmStep::qset): GPU suite, then same-box A/B PM_QSET=0 vs 1
# on the serving bench (kernel averages and q/s), alternating.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
F="--steps 60 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single"
for i in 1 2; do
  for q in 0 1; do
    PM_QSET=$q timeout -k 10 300 python -u bench.py $F > gpurun_out/qs_$q-$i.json 2>/dev/null || exit 1
    python -c "
import json
d=json.load(open('gpurun_out/qs_$q-$i.json')); k=d['kernel_avg_us']; iso=d['isolated']['kernel_avg_us']; m=d.get('config2_private_search',{})
print('qset=$q', d['value'], 'answer', k['answer'], 'mr', k['match_resolve'], 'iso answer', iso['answer'], 'iso mr', iso['match_resolve'], 'msm', m.get('private_queries_per_s'), m.get('kernel_avg_us',{}).get('answer'))"
  done
done
