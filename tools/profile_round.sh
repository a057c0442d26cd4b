# Profile set of one round on one MI355X (run through gpurun from the repo root),
# one stage per gpurun call:
#   bench   bench.json: the bench line (the driver's command)
#   trace   rocprofv3 --kernel-trace --stats of the same bench (no cpu_baseline)
#   pmcf    rocprofv3 --pmc FETCH_SIZE   (separate passes of the same command)
#   pmcw    rocprofv3 --pmc WRITE_SIZE
# usage: bash tools/profile_round.sh OUTDIR STAGE...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
B="bench.py --steps 20 --warmup 5"
for st in "$@"; do
  case $st in
    bench) timeout -k 10 900 python3 $B > $OUT/bench.json 2> $OUT/bench.err || exit 1 ;;
    trace) timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B --no-cpu-baseline > $OUT/bench_trace.json 2> $OUT/trace.err || exit 1 ;;
    pmcf) timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmcf -o run -- python3 $B --no-cpu-baseline > $OUT/bench_pmcf.json 2> $OUT/pmcf.err || exit 1 ;;
    pmcw) timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmcw -o run -- python3 $B --no-cpu-baseline > $OUT/bench_pmcw.json 2> $OUT/pmcw.err || exit 1 ;;
  esac
done
find $OUT -name "*.csv" -size +1M -exec gzip -f {} \;
find $OUT -type f | head -40
