#!/bin/bash
out=gpurun_out/r03pool2
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_fullsize.py -k "sessions_batched or sift1m_full_sessions" > $out/tests.log 2>&1
rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
B="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-single --no-bigann --no-config0 --no-msmarco-search"
for i in 1 2; do
  PM_TEAM_TRACE=$PWD/$out/trace$i.csv timeout -k 10 200 python -u bench.py $B > $out/pool$i.json 2>> $out/err.log || exit 1
  PM_BATCH_POOL=0 timeout -k 10 200 python -u bench.py $B > $out/team$i.json 2>> $out/err.log || exit 1
done
for f in $out/pool1.json $out/team1.json $out/pool2.json $out/team2.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
