"""Diagnostic: where one client's TestBatchPIRPerf batch (bench.py configs[2])
spends its wall time: Python call, host step phases, the k_step kernel.

    python tools/batchpir_host.py [batches]

Prints per-batch means (us) of the wall time of g.Query, the library's
host_batch_query (C entry to return), its launch / wait / post phases, the
first-token and all-token waits, and the step kernel's event time, with the
step timing off (wall only) and on (level 2, as bench.py runs it).
"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))


def main(batches=300):
    import pacmann_amd as pm
    N, E, B = 3_201_821, 112, 32
    db = np.random.default_rng(77).integers(0, 2**64, size=N * E, dtype=np.uint64)
    ctx = pm.Context(0)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=21, ctx=ctx)
    g.Preprocessing()
    ctx.sync()
    rng = np.random.default_rng(78)
    ids = rng.integers(0, N, size=(3 * batches + 20, B)).astype(np.uint64)
    for b in ids[:20]:
        g.Query(b)
    ctx.sync()
    keys = ["host_batch_query", "host_step_launch", "host_step_wait", "host_step_post",
            "host_wait_first_token", "host_wait_all_tokens", "host_wait_done"]
    for level, sl in ((0, slice(20, 20 + batches)), (2, slice(20 + batches, 20 + 2 * batches)),
                      (1, slice(20 + 2 * batches, 20 + 3 * batches))):
        ctx.timing_reset()
        ctx.timing(level)
        t0 = time.perf_counter()
        for b in ids[sl]:
            g.Query(b)
        ctx.sync()
        wall = (time.perf_counter() - t0) / batches * 1e6
        ctx.timing(0)
        line = f"timing {level}: wall {wall:7.2f} us/batch"
        for k in keys + ["step"]:
            n, ms, _ = ctx.timing_get(k)
            if n:
                line += f"  {k.replace('host_', '')} {ms / batches * 1e3:6.2f}" + (f" (n {n})" if n != batches else "")
        print(line, flush=True)
    # the bare Python / ctypes cost of a call that fails at argument checking
    out = np.zeros((B, E), dtype=np.uint64)
    t0 = time.perf_counter()
    for _ in range(batches):
        np.zeros((B, E), dtype=np.uint64)
        pm._u64(ids[0]).ravel()
    print(f"python marshalling alone: {(time.perf_counter() - t0) / batches * 1e6:.2f} us/batch", flush=True)
    del out


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 300)
