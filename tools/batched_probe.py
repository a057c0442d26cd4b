"""Throughput of batched multi-session serving on the SIFT1M-shaped bench data.

    python tools/batched_probe.py --sessions 8 16 32 --queries 40 [--threads 16]

Builds the bench's data (SIFT-like vectors, GPU-built graph), one server, and
for each S: S client sessions served by pm_search_loop_batched; prints q/s.
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import pacmann_amd as pm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sessions", type=int, nargs="+", default=[8, 16])
ap.add_argument("--queries", type=int, default=40)
ap.add_argument("--threads", type=int, default=0)
ap.add_argument("--groups", type=int, default=1)
ap.add_argument("--timing", type=int, default=0)
a = ap.parse_args()
ctx0 = pm.Context(0)
v, g, _ = bench.make_data(0, "built", ctx0)
base = pm.PIRGraphInfo(v, g, pir_seed=11, search_seed=12, ctx=ctx0)
base.Preprocess()
for S in a.sessions:
    sess = [base.Session(100 + i, 200 + i) for i in range(S)]
    for s in sess:
        s.Preprocess()
    qs = bench.make_queries(v, S * (a.queries + 2), seed=300).reshape(S, a.queries + 2, -1)
    pm.search_loop_batched(sess, qs[:, :2], bench.K_TOP, bench.STEP, bench.PARALLEL, a.groups, a.threads)   # warm-up
    for s in sess:
        s.ctx.timing_reset()
        s.ctx.timing(a.timing)
    t0 = time.perf_counter()
    ans, wall, on, mt = pm.search_loop_batched(sess, qs[:, 2:], bench.K_TOP, bench.STEP, bench.PARALLEL, a.groups,
                                               a.threads)
    el = time.perf_counter() - t0
    out = {"S": S, "groups": a.groups, "threads": a.threads, "queries_per_s": round(S * a.queries / wall, 1), "wall_s": round(wall, 4),
           "ms_per_round": round(wall / a.queries / bench.STEP * 1e3, 4), "maint_s_mean": round(float(mt.mean()), 4)}
    if a.timing:
        c = sess[0].ctx
        out["kernels_us"] = {k: round(c.timing_get(k)[1] / max(c.timing_get(k)[0], 1) * 1e3, 2)
                             for k in ("hint_match", "resolve", "match_resolve", "gather", "answer", "prep_offsets", "prep_fold")}
        for hname in ("host_step_launch", "host_step_wait", "host_step_post", "host_batch_query", "host_knn_update",
                      "host_gvi_parse", "host_knn_init"):
            n, ms, _ = c.timing_get(hname)
            out.setdefault("host_us_per_call_s0", {})[hname] = round(ms / max(n, 1) * 1e3, 2)
    print(json.dumps(out), flush=True)
    del sess
