# Replacement rows hashed once per row (k_prep_repl): GPU suite, then a
# same-box A/B against the previous commit (build/libpacmann_prev.so).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
F="--steps 60 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for i in 1 2; do
  for v in prev head; do
    if [ $v = head ]; then L=""; else L="PM_LIB=$PWD/build/libpacmann_$v.so"; fi
    env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/rp_$v-$i.json 2>/dev/null || exit 1
    python tools/ab_summary.py gpurun_out/rp_$v-$i.json
  done
done
