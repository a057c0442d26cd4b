# k_answer_s workgroup size with 6-row batches (PM_ANSWER_NT 128 default / 256): serving bench, mirrored order.
set -o pipefail
mkdir -p gpurun_out
F="--steps 40 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for nt in 128 256 256 128; do
  PM_ANSWER_NT=$nt timeout -k 10 300 python -u bench.py $F > gpurun_out/nt_$nt.json 2>/dev/null || exit 1
  python tools/ab_summary.py gpurun_out/nt_$nt.json
done
