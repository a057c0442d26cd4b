# One-round-trip match+resolve (k_match_resolve_s): GPU suite, then A/B of batched
# serving (PM_MATCH_RESOLVE=1 default: k_match_resolve_s; 2: the general k_match_resolve).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
F="--steps 40 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single"
for i in 1 2; do
  timeout -k 10 400 python -u bench.py $F > gpurun_out/mrs_on$i.json 2>/dev/null || exit 1
  PM_MATCH_RESOLVE=2 timeout -k 10 400 python -u bench.py $F > gpurun_out/mrs_off$i.json 2>/dev/null || exit 1
  python -c "
import json
for n in ['mrs_on$i','mrs_off$i']:
    d=json.load(open(f'gpurun_out/{n}.json')); m=d.get('config2_private_search') or {}
    print(n, d['value'], d['kernel_avg_us'], d.get('isolated',{}).get('kernel_avg_us'), 'msmarco', m.get('private_queries_per_s'), m.get('kernel_avg_us'))"
done
