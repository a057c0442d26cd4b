# Where the fold's cycles go: one --pmc pass (8 SQ counters) over the serving bench.
set -o pipefail
mkdir -p gpurun_out/foldpmc
export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/foldpmc -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search > gpurun_out/foldpmc/bench.json 2> gpurun_out/foldpmc/err.log || { tail -5 gpurun_out/foldpmc/err.log; exit 1; }
python - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open('gpurun_out/foldpmc/run_counter_collection.csv')):
    k = (r['Kernel_Name'][:40], int(r['Grid_Size']))
    acc[k][r['Counter_Name']] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
for k, c in acc.items():
    if not any(x in k[0] for x in ('fold_rot', 'answer_s', 'match_resolve_s', 'prep_offsets')): continue
    w = c['SQ_WAVE_CYCLES'] or 1
    print(k, {x: round(v / w, 3) for x, v in c.items() if x != 'SQ_WAVE_CYCLES'}, 'wave_cycles', int(w))
PY
gzip -f gpurun_out/foldpmc/run_counter_collection.csv
