"""Probe: S client sessions over one graph and server DB on one GPU
(pm_search_loop_sessions: one host thread and stream per session).

    python tools/multi_session.py S_MAX [queries_per_session]

Prints aggregate queries/s for S = 1..S_MAX.
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
import pacmann_amd as pm  # noqa: E402

smax = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 100
v, g, _ = bench.make_data(0, "random", None)
qs = bench.make_queries(v, smax * nq + 8, seed=300)
base = pm.PIRGraphInfo(v, g, pir_seed=11, search_seed=12, ctx=pm.Context(0))
base.Preprocess()
sess = [base.Session(11 + s, 12 + s) for s in range(smax)]
for s in sess:
    s.Preprocess()
pm.search_loop_sessions(sess, np.stack([qs[:3]] * smax), 10, 20, 3)
print("sessions ready", flush=True)
for S in range(1, smax + 1):
    q = qs[8:8 + S * nq].reshape(S, nq, -1)
    _, wall, on, mt = pm.search_loop_sessions(sess[:S], q, 10, 20, 3)
    print(f"S={S}: aggregate {S * nq / wall:.1f} q/s, per-session {[round(nq / (a + b), 1) for a, b in zip(on, mt)]}",
          flush=True)
