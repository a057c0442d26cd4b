out=${OUT:-gpurun_out/sweep_s}; mkdir -p $out
B="--no-cpu-baseline --no-config2 --no-config0 --no-msmarco-search --no-bigann --no-single"
for n in ${SWEEP:-256 320 384 288 288 384 320 256}; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 $B --sessions $n > $out/s$n.json 2>> $out/err.log || exit 1
  python tools/ab_summary.py sift "S=$n" $out/s$n.json | tee -a $out/summary.log
done
