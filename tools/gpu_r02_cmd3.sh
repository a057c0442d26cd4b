set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "hub or build_graph" > gpurun_out/hub.log 2>&1 || { tail -30 gpurun_out/hub.log; exit 1; }
tail -3 gpurun_out/hub.log
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-kernel-timing --no-cpu-baseline --no-config2 --no-msmarco-search --no-config0 --no-bigann > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-msmarco-search --no-config0 --no-bigann > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err || exit 1
