mkdir -p gpurun_out
for a in "--groups 4 --threads 4" "--groups 4 --threads 8" "--groups 4 --threads 12" "--groups 4 --threads 16" "--groups 2 --threads 8" "--groups 3 --threads 12"; do
  timeout -k 10 200 python -u tools/batched_probe.py --sessions 128 --queries 15 $a >> gpurun_out/ab.log 2>&1 || exit 1
done
nproc >> gpurun_out/ab.log
python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/ab.log
