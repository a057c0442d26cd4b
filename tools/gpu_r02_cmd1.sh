set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gputests.log; exit 1; }
tail -3 gpurun_out/gputests.log
for v in pub0 default pub2; do
  if [ $v = default ]; then L=pacmann_amd/libpacmann.so; else L=build/libpacmann_$v.so; fi
  PM_LIB=$L PM_ROWS_CHECK=2 timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --graph random > gpurun_out/audit_$v.json 2> gpurun_out/audit_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/audit_$v.json'));print('$v', d['value'], d['rows_check'], d['roofline']['avg_ms'])"
done
