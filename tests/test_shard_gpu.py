"""The sharded batch PIR with real libpacmann.so shards and the device-resident
combine (pacmann_amd/shard.py; sharding axis batch-pir.go:62-85).

* world 2 over gloo: two processes on cuda:0 (the GPU box has one GPU), each
  holding half of the 16 partitions in its own HIP context; the responses go
  device-to-device into one tensor per rank (pm_batchpir_query_dev), which
  the gloo collective sums.  Both ranks' combined answers and flags must equal
  an unsharded oracle run, batch by batch, through the batch layer's
  re-preprocessing trigger.
* world 1 over nccl (RCCL): the same device tensor all-reduced in place by
  RCCL on torch's stream — the code path the multi-GPU bench runs at N > 1,
  with the one rank a gpurun box allows.

Multi-GPU RCCL over xGMI (N = 2..8) is not runnable here (one GPU per box):
unmeasured on hardware, correct by construction of these two paths."""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, E, B, F, SEED = 60_000, 12, 16, 8, 4321


def _db():
    return np.random.default_rng(13).integers(0, 2**64, size=N * E, dtype=np.uint64)


def _batches(n, wide=False):
    """3B ids per batch (6 sub-queries per partition), or with wide=True 6B
    (12 per partition) whose first 16 ids are new ids of partition 0 spread
    over its chunks (no per-chunk limit, pir.go:396-400): that
    partition's FinishedQueryNum then tracks QueriesMadeInPartition, so late
    in the window a batch would take it past MaxQueryNum and the engine serves
    it by the multi-step path (one sub-query at a time, pir.go:527-530)."""
    rng = np.random.default_rng(14)
    PS = N // (B // 2)
    for b in range(n):
        if wide:   # partition 0: 16 ids never asked before (no local-cache hits); the rest elsewhere
            q = rng.integers(PS, N, size=6 * B, dtype=np.uint64)
            q[:16] = (np.arange(b * 16, b * 16 + 16, dtype=np.uint64) * np.uint64(263)) % np.uint64(PS)   # spread over chunks
        else:
            q = rng.integers(0, N, size=3 * B, dtype=np.uint64)
            q[4] = q[1]
        yield q


def _nbatches(wide=False):
    from oracle import oracle as O
    o = O.PianoPIR(N // (B // 2), E * 8, np.zeros(N // (B // 2) * E, np.uint64), F)
    return int(o.Config()["MaxQueryNum"] // (6 if wide else 3)) + 6   # past the re-preprocessing trigger


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir, backend, nb, wide):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from pacmann_amd.shard import ShardedBatchPIR
        pir = ShardedBatchPIR(N, E * 8, B, _db(), F, seed=SEED, device=0)
        assert pir.device_path and pir.pir.nshards == world and pir.pir.shard == rank
        pir.Preprocessing()
        rows, oks = [], []
        for q in _batches(nb, wide):
            dev = pir.QueryDevice(q)
            assert dev.is_cuda and dev.shape == (len(q), E + 1)
            h = dev.cpu().numpy().view(np.uint64)
            rows.append(h[:, :E].copy())
            oks.append(h[:, E].copy())
        np.save(os.path.join(out_dir, f"rows{rank}.npy"), np.stack(rows))
        np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.stack(oks))
        steps = pir.pir.ctx.timing_get("host_step_launch")[0]   # steps run (a multi-step batch runs several)
        np.save(os.path.join(out_dir, f"prep{rank}.npy"), np.array([pir.stats()["PrepCount"], steps]))
    finally:
        dist.destroy_process_group()


def _run(world, backend, oracle, wide=False):
    import torch.multiprocessing as mp
    nb = _nbatches(wide)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(world, _free_port(), d, backend, nb, wide), nprocs=world, join=True)
        rows = [np.load(os.path.join(d, f"rows{r}.npy")) for r in range(world)]
        oks = [np.load(os.path.join(d, f"ok{r}.npy")) for r in range(world)]
        preps = [int(np.load(os.path.join(d, f"prep{r}.npy"))[0]) for r in range(world)]
        steps = [int(np.load(os.path.join(d, f"prep{r}.npy"))[1]) for r in range(world)]
    for r in range(1, world):   # every rank holds the combined answer
        assert np.array_equal(rows[r], rows[0]) and np.array_equal(oks[r], oks[0])
    db = _db()
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, F, seed=SEED)
    o.Preprocessing()
    full = db.reshape(N, E)
    for i, q in enumerate(_batches(nb, wide)):
        want, _ = o.Query(q)
        assert np.array_equal(rows[0][i], want), i
        ok = oks[0][i].astype(bool)
        assert set(np.unique(oks[0][i]).tolist()) <= {0, 1}
        assert np.array_equal(rows[0][i][ok], full[q.astype(np.int64)][ok]), i
        assert not rows[0][i][~ok].any(), i
    assert preps[0] == o.stats()["PrepCount"] > 1
    if wide:   # rank 0 holds partition 0: some batch took the multi-step path there
        assert steps[0] > nb, (steps[0], nb)


def test_sharded_device_combine_gloo_world2(oracle):
    _run(2, "gloo", oracle)


def test_sharded_device_combine_rccl_world1(oracle):
    _run(1, "nccl", oracle)


def test_sharded_device_combine_multistep_gloo_world2(oracle):
    """The same combine when a batch takes partition 0 past its query budget
    mid-batch: the owning rank's rows come from the multi-step path (staged on
    the host, copied to the device tensor in stream order)."""
    _run(2, "gloo", oracle, wide=True)
