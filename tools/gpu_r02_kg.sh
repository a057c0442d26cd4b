# k_answer rows per thread in flight (PM_ANSWER_KG 6 / 8 default / 10): the parity subset of the
# batched path on each build, then the serving bench's answer times, mirrored order.
set -o pipefail
mkdir -p gpurun_out
for v in kg6 kg10; do
  PM_LIB=$PWD/build/libpacmann_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q -k shared_step --timeout 500 --timeout-method thread > gpurun_out/kg_$v.log 2>&1 || { echo FAILED $v; tail -5 gpurun_out/kg_$v.log; exit 1; }
  tail -1 gpurun_out/kg_$v.log
done
F="--steps 40 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for v in kg6 head kg10 kg10 head kg6; do
  if [ $v = head ]; then L=""; else L="PM_LIB=$PWD/build/libpacmann_$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/kgb_$v.json 2>/dev/null || exit 1
  python tools/ab_summary.py gpurun_out/kgb_$v.json
done
