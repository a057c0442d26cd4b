#!/bin/bash
# Same-box A/B of builds or environment switches, in ABBA order (the variants,
# then the same list reversed: cancels drift between consecutive runs on one box).
#
# usage: tools/ab.sh OUTDIR WORKLOAD VARIANT...
#   WORKLOAD  sift     bench.py, SIFT1M serving block only (one line per run: q/s, step and maintenance kernels)
#             bigann   bench.py, BIGANN-100M / 1B blocks only (q/s, ms per round, step kernels)
#             probe    tools/batched_probe.py: 64 sessions in one lock-step group alone, kernel averages
#             fold     tools/group_fold_probe.py 64 4: the 64-client SIFT1M group fold
#             fold1    tools/fold_probe.py: one client's preprocessing kernels
#   VARIANT   default | path/to/lib.so (PM_LIB) | VAR=value[,VAR=value...] (environment)
#   env       TESTS="pytest -k expression": the parity subset first, on the product build
#             ARGS="...": extra arguments for the workload's program
# Each run appends to OUTDIR/summary.log; the raw outputs stay in OUTDIR.
out=$1; wl=$2; shift 2
mkdir -p "$out"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_fullsize.py tests/test_shard_search_gpu.py -k "$TESTS" > "$out/tests.log" 2>&1
  rc=$?; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
fi
B="--no-cpu-baseline --no-config2 --no-config0 --no-msmarco-search"
vars=("$@"); rev=(); for ((i=${#vars[@]}-1; i>=0; i--)); do rev+=("${vars[$i]}"); done
n=0
for v in "${vars[@]}" "${rev[@]}"; do
  n=$((n+1))
  envs=()
  case $v in
    default) ;;
    *.so) envs=("PM_LIB=$PWD/$v") ;;
    *=*) IFS=, read -ra envs <<< "$v" ;;
    *) echo "bad variant $v"; exit 2 ;;
  esac
  f=$out/run$n
  case $wl in
    sift) env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $B --no-bigann $ARGS > $f.json 2>> $out/err.log || exit 1
          python tools/ab_summary.py sift "$v" $f.json | tee -a "$out/summary.log" ;;
    bigann) env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $B --no-single $ARGS > $f.json 2>> $out/err.log || exit 1
          python tools/ab_summary.py bigann "$v" $f.json | tee -a "$out/summary.log" ;;
    probe) env "${envs[@]}" timeout -k 10 300 python -u tools/batched_probe.py --sessions 64 --queries 6 --timing 2 $ARGS > $f.log 2>&1 || exit 1
          { echo "== $v"; tail -4 $f.log; } | tee -a "$out/summary.log" ;;
    fold) env "${envs[@]}" timeout -k 10 300 python -u tools/group_fold_probe.py ${ARGS:-64 4} > $f.log 2>&1 || exit 1
          { echo "== $v"; grep prep_fold $f.log; } | tee -a "$out/summary.log" ;;
    fold1) env "${envs[@]}" timeout -k 10 120 python -u tools/fold_probe.py $ARGS > $f.log 2>&1 || exit 1
          { echo "== $v"; tail -4 $f.log; } | tee -a "$out/summary.log" ;;
    *) echo "bad workload $wl"; exit 2 ;;
  esac
done
