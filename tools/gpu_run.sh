#!/bin/bash
# One GPU-box session: the -m gpu suite (or a subset), smoke and the default
# bench line, each step under its own time limit; stops at the first step that
# crashed, faulted or timed out (pytest's exit 1 = test failures: continue).
# usage: tools/gpu_run.sh OUTDIR [pytest-args...]   (env: BENCH_ARGS, NO_BENCH=1, NO_TESTS=1)
out=${1:-gpurun_out/run}; shift
mkdir -p "$out"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread --maxfail=5 "${@:-tests}" \
    > "$out/gputests.log" 2>&1
  rc=$?
  tail -3 "$out/gputests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
  rc=$?; tail -2 "$out/smoke.log"
  if [ $rc -ne 0 ]; then echo "smoke rc=$rc: stopping"; exit $rc; fi
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > "$out/bench.json" 2> "$out/bench.err"
  rc=$?; tail -c 600 "$out/bench.json"; tail -3 "$out/bench.err"
  exit $rc
fi
