"""Diagnostic: the sharded batch-PIR sequence of tests/test_gpu_parity.py::
test_batch_pir_shards, repeated over several seeds; on the first mismatch it
prints which ids differ, the owning shard, its mask and the first sub-queries'
state.  PM_NO_FUSE=1 runs the three-kernel path."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import pacmann_amd as pm  # noqa: E402
from oracle import oracle as O  # noqa: E402

SEED = 20240501


def run(nshards, dbseed, qseed, N=30_000, E=6, B=8):
    db = np.random.default_rng(dbseed).integers(0, 2**64, size=N * E, dtype=np.uint64)
    ctx = pm.default_context()
    shards = [pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx, shard=r, nshards=nshards)
              for r in range(nshards)]
    o = O.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED)
    for s in shards:
        s.Preprocessing()
    o.Preprocessing()
    P = shards[0].Config()["PartitionNum"]
    PS = shards[0].Config()["PartitionSize"]
    rng = np.random.default_rng(qseed)
    maxq = shards[0].SubConfig(0)["MaxQueryNum"]
    for b in range(int(maxq // 3) + 6):
        q = rng.integers(0, N, size=3 * B, dtype=np.uint64)
        q[4] = q[1]
        parts = [s.QueryWithMask(q) for s in shards]
        got = sum(p[0] for p in parts)
        want, _ = o.Query(q)
        if not np.array_equal(got, want):
            bad = np.where((got != want).any(axis=1))[0]
            print(f"MISMATCH nshards={nshards} db={dbseed} q={qseed} batch={b}: ids {bad.tolist()}")
            for i in bad[:6]:
                part = int(q[i]) // PS
                sh = part % nshards
                print(f"  id {int(q[i])} part {part} shard {sh} ok={[bool(p[1][i]) for p in parts]} "
                      f"got0={int(got[i][0])} want0={int(want[i][0])} rows_equal_db={bool((want[i] == db.reshape(N, E)[int(q[i])]).all())}")
            return False
    return True


if __name__ == "__main__":
    fails = 0
    for nsh in (3, 2):
        for seed in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
            ok = run(nsh, 77 + seed, 11 + seed)
            fails += not ok
            print(f"nshards={nsh} seed={seed}: {'ok' if ok else 'FAIL'}", flush=True)
    print("fails", fails)
