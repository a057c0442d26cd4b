mkdir -p gpurun_out
for a in "--sessions 256 --groups 4 --threads 16" "--sessions 384 --groups 4 --threads 16" "--sessions 512 --groups 4 --threads 16" "--sessions 384 --groups 6 --threads 16"; do
  timeout -k 10 250 python -u tools/batched_probe.py --queries 46 $a >> gpurun_out/ab.log 2>&1 || exit 1
done
