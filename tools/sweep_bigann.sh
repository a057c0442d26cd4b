#!/bin/bash
# BIGANN blocks of the bench over serving settings (team count, host threads), in the given order.
# usage: tools/sweep_bigann.sh OUTDIR "ARGS1" "ARGS2" ...   (env TESTS: parity subset first)
out=$1; shift; mkdir -p $out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_shard_search_gpu.py -k "$TESTS" > $out/tests.log 2>&1
  rc=$?; tail -2 $out/tests.log; [ $rc -eq 0 ] || exit $rc
fi
B="--steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-config0 --no-msmarco-search --no-single"
for a in "$@"; do
  timeout -k 10 300 python -u bench.py $B $a > $out/b.json 2>> $out/err.log || exit 1
  python tools/ab_summary.py bigann "$a" $out/b.json | tee -a $out/summary.log
done
