"""BIGANN-scale batch PIR probe (BASELINE.json configs[3]/[4]) on one GPU.

    python tools/bigann_probe.py N [--E 80] [--shard s --nshards n] [--steps 40] [--ids 96]

Device-generated DB (pm_batchpir_create_synth), one full preprocessing with
per-kernel times, then `steps` batch queries of `ids` uniform ids with the
reference's property check (every successful entry == its DB row, recomputed
on the host from the synth spec).
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import pacmann_amd as pm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("N", type=int)
ap.add_argument("--E", type=int, default=80)
ap.add_argument("--shard", type=int, default=0)
ap.add_argument("--nshards", type=int, default=1)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--ids", type=int, default=96)
ap.add_argument("--preps", type=int, default=1)
a = ap.parse_args()

ctx = pm.Context(0)
ctx.timing(2)
t0 = time.time()
g = pm.SimpleBatchPianoPIR(a.N, a.E * 8, 32, None, 8, seed=5, ctx=ctx, shard=a.shard, nshards=a.nshards,
                           db_seed=11)
t_create = time.time() - t0
cfg = g.SubConfig(a.shard)
print("subconfig", cfg, "create_s", round(t_create, 2), flush=True)
for i in range(a.preps):
    ctx.timing_reset()
    t0 = time.time()
    g.Preprocessing()
    ctx.sync()
    tp = time.time() - t0
    ks = {k: ctx.timing_get(k) for k in ("prep_init", "prep_offsets", "prep_fold", "prep_repl")}
    print("prep", i, round(tp, 4), json.dumps(ks), flush=True)
rng = np.random.default_rng(3)
ctx.timing_reset()
bad = nok = 0
t0 = time.time()
for s in range(a.steps):
    ids = rng.integers(0, a.N, size=a.ids).astype(np.uint64)
    out, ok = g.QueryWithMask(ids)
    sel = np.where(ok)[0]
    nok += len(sel)
    if len(sel):
        want = pm.synth_rows(11, ids[sel], a.E)
        bad += int((out[sel] != want).any(axis=1).sum())
tq = time.time() - t0
ks = {k: ctx.timing_get(k) for k in ("step", "hint_match", "resolve", "gather", "answer")}
print("query steps", a.steps, "s", round(tq, 4), "ms/step", round(1e3 * tq / a.steps, 3), "ok", nok, "bad", bad,
      json.dumps(ks), flush=True)
print("stats", g.stats(), flush=True)
