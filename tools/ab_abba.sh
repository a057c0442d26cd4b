# Same-box A/B in ABBA order (cancels drift between consecutive runs) of the serving bench:
#   bash tools/ab_abba.sh NAME_A LIB_A NAME_B LIB_B   (LIB "-" = the in-tree libpacmann.so)
set -o pipefail
mkdir -p gpurun_out
F="--steps 60 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
run() {
  if [ "$2" = "-" ]; then L=""; else L="PM_LIB=$PWD/$2"; fi
  env $L timeout -k 10 300 python -u bench.py $F > gpurun_out/abba_$1-$3.json 2>/dev/null || exit 1
  python tools/ab_summary.py gpurun_out/abba_$1-$3.json
}
run $1 $2 1 && run $3 $4 1 && run $3 $4 2 && run $1 $2 2
