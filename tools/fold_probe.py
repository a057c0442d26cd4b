# Diagnostic: average k_prep_fold* time of a SIFT1M-shaped batch PIR
# preprocessing (16 partitions, E = 80).  PM_LIB selects a diagnostic build.
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pacmann_amd as pm
N, E, B = 1_000_000, 80, 32
db = np.random.default_rng(0).integers(0, 2**64, size=N * E, dtype=np.uint64)
ctx = pm.Context(0)
g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=1, ctx=ctx)
g.Preprocessing()
ctx.timing_reset()
ctx.timing(True)
for _ in range(8):
    g.Preprocessing()
ctx.timing(False)
for k in ("prep_offsets", "prep_fold", "prep_repl"):
    n, ms, by = ctx.timing_get(k)
    print(f"{os.environ.get('PM_LIB', 'default')} {k}: {ms / max(n, 1):.4f} ms/launch over {n}", flush=True)
