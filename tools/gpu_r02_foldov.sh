# Fold staging overlap: GPU suite on the tree, then the one-client and 64-client fold times of
# the committed build (prev), the deferred kSkip select without the L2 prefetch (pf0) and the tree
# (deferred select + prefetch), in mirrored order.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
F="--steps 40 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for v in prev pf0 head head pf0 prev; do
  if [ $v = head ]; then L=""; else L="PM_LIB=$PWD/build/libpacmann_$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/fo_$v.json 2>/dev/null || exit 1
  python -c "
import json
d=json.load(open('gpurun_out/fo_$v.json')); k=d['kernel_avg_us']
print('$v', d['value'], 'fold64', k['prep_fold'], 'iso fold1', d['isolated']['kernel_avg_us']['prep_fold_one_client'], 'answer', k['answer'])"
done
