# Current-tree check on one MI355X: the whole -m gpu suite, smoke, then the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/gputests.log | head -20; tail -5 gpurun_out/gputests.log; exit 1; }
tail -2 gpurun_out/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -20 gpurun_out/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));print(d['value'], d['roofline'])"
