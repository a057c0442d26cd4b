"""Diagnostic: one client's preprocessing of a BIGANN-shaped shard (synthetic
DB generated on the device): per-kernel device time of k_prep_offsets and the
fold.  usage: python tools/fold_wide_probe.py [100m|1b] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import pacmann_amd as pm

shape = sys.argv[1] if len(sys.argv) > 1 else "100m"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
N, ns = (100_000_000, 1) if shape == "100m" else (1_000_000_000, 8)
ctx = pm.Context(0)
g = pm.SimpleBatchPianoPIR(N, 640, 32, None, 8, seed=1, ctx=ctx, shard=0, nshards=ns, db_seed=41)
g.Preprocessing()
ctx.timing_reset()
ctx.timing(True)
for _ in range(reps):
    g.Preprocessing()
ctx.timing(False)
for k in ("prep_offsets", "prep_fold", "prep_repl"):
    n, ms, by = ctx.timing_get(k)
    print(f"{shape} {os.environ.get('PM_FOLD_WIDE', '1')} {k}: {ms / max(n, 1):.3f} ms/launch over {n}"
          + (f", {by / n / (ms / n / 1e3) / 1e12:.2f} T units/s" if n and ms else ""), flush=True)
