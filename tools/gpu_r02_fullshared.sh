# Full-size shared-step parity (the bench's kernels), at the default resolver size and at PM_MR_NT=128,
# then a same-box A/B of the two resolver sizes.
set -o pipefail
mkdir -p gpurun_out
K="shared_step"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -k $K --timeout 500 --timeout-method thread > gpurun_out/fs256.log 2>&1 || { echo FAILED256; grep -E "FAILED|Error|assert" gpurun_out/fs256.log | head -20; tail -5 gpurun_out/fs256.log; exit 1; }
tail -1 gpurun_out/fs256.log
PM_MR_NT=128 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -k $K --timeout 500 --timeout-method thread > gpurun_out/fs128.log 2>&1 || { echo FAILED128; grep -E "FAILED|Error|assert" gpurun_out/fs128.log | head -20; tail -5 gpurun_out/fs128.log; exit 1; }
tail -1 gpurun_out/fs128.log
F="--steps 60 --warmup 5 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
for i in 1 2; do
  for nt in 256 128; do
    PM_MR_NT=$nt timeout -k 10 300 python -u bench.py $F > gpurun_out/mr_$nt-$i.json 2>/dev/null || exit 1
    python tools/ab_summary.py gpurun_out/mr_$nt-$i.json
  done
done
