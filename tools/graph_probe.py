"""Probe: GPU graph build + kNN ground truth at bench scale, and recall of the
non-private search over the built graph vs the random graph.

    python tools/graph_probe.py N [queries]
"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import pacmann_amd as pm  # noqa: E402
from pacmann_amd.report import compute_recall  # noqa: E402
from pacmann_amd.synth import random_graph, sift_like_vectors  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 100
v = sift_like_vectors(n, 128, seed=100)
ctx = pm.Context(0)
t = time.perf_counter()
g, tm = pm.build_graph(v, 32, 1.2, seed=1, ctx=ctx)
print(f"build_graph n={n}: {time.perf_counter() - t:.2f}s {tm}", flush=True)
qs = bench.make_queries(v, nq, seed=300)
t = time.perf_counter()
gt = pm.knn(v, qs, 10, ctx)
print(f"knn gt {nq} queries: {time.perf_counter() - t:.3f}s", flush=True)
for name, gg in [("built", g), ("random", random_graph(n, 32, seed=200))]:
    gi = pm.PIRGraphInfo(v, gg, nonprivate=True, pir_seed=1, search_seed=2, ctx=ctx)
    gi.Preprocess()
    ans, _, _ = gi.SearchLoop(qs, 10, 20, 3)
    print(f"{name} graph: non-private recall@10 {compute_recall(gt, ans, 10):.4f}", flush=True)
