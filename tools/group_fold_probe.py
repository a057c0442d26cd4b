"""The serving loop's maintenance fold at the bench's group shape: K SIFT1M
clients (1e6 x 640 B) preprocessed as ONE launch set
(pm_batchpir_group_preprocessing); prints the per-launch kernel times.
PM_LIB selects a diagnostic build.

    python tools/group_fold_probe.py [K] [reps] [sift1m|msmarco]
"""
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import pacmann_amd as pm  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
shape = sys.argv[3] if len(sys.argv) > 3 else "sift1m"
N, E, B = (1_000_000, 80, 32) if shape == "sift1m" else (3_201_821, 112, 32)
db = np.random.default_rng(0).integers(0, 2**64, size=N * E, dtype=np.uint64)
ctx = pm.Context(0)
server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=1, ctx=ctx)
server.Preprocessing()
cg = pm.Context(0)
cl = [server.Client(100 + i, cg) for i in range(K)]
for c in cl:
    c.Preprocessing()
grp = pm.BatchPIRGroup(cl)
grp.Preprocessing()   # warm-up
cg.timing_reset()
cg.timing(True)
for _ in range(reps):
    grp.Preprocessing()
cg.timing(False)
tag = os.path.basename(os.environ.get("PM_LIB", "default"))
for k in ("prep_offsets", "prep_fold", "prep_repl"):
    n, ms, by = cg.timing_get(k)
    print(f"{tag} {shape} K={K} {k}: {ms / max(n, 1):.3f} ms/launch over {n}", flush=True)
