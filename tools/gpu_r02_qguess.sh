# k_match_resolve_s: query-set tiles guessed and loaded by waves 1.. during wave 0's chain:
# GPU suite, then the kernels alone and among the groups vs the committed build, mirrored order.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
F="--steps 40 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for v in prev head head prev; do
  if [ $v = head ]; then L=""; else L="PM_LIB=$PWD/build/libpacmann_$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/qg_$v.json 2>/dev/null || exit 1
  python tools/ab_summary.py gpurun_out/qg_$v.json
done
