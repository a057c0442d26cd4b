set -o pipefail
for v in pub3 pub0 pub3; do
  L=build/libpacmann_$v.so
  PM_LIB=$L PM_ROWS_CHECK=2 timeout -k 10 300 python -u bench.py --steps 100 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --graph random > gpurun_out/audit_$v.json 2> gpurun_out/audit_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/audit_$v.json'));print('$v', d['value'], d['rows_check'], d['roofline']['avg_ms'])"
done
