# one client's TestBatchPIRPerf loop, product build vs another build (PM_LIB), ABBA
# usage: bash tools/step_ab_lib.sh OUTDIR path/to/other.so
out=$1; other=$2; mkdir -p $out
for v in new base base new; do
  echo "== $v" >> $out/host.log
  if [ $v = base ]; then PM_LIB=$PWD/$other timeout -k 10 300 python -u tools/batchpir_host.py 300 >> $out/host.log 2>&1 || exit 1
  else timeout -k 10 300 python -u tools/batchpir_host.py 300 >> $out/host.log 2>&1 || exit 1; fi
done
