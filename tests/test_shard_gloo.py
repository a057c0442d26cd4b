"""Multi-rank (world_size 2, gloo, CPU) test of the partition-sharded batch PIR
combine (pacmann_amd/shard.py).

Each rank's shard engine is the oracle restricted to the partitions the rank
owns (p % world == rank): the test checks the distributed glue, not the GPU
shard itself. The summed, all-reduced entries must equal an unsharded oracle
run on the same batches. test_gpu_parity.py::test_batch_pir_shards checks the
C engine's own shards on the GPU."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

N, E, B, F, SEED = 20_000, 4, 8, 8, 1234


class OracleShard:
    """Oracle SimpleBatchPianoPIR answering only the owned partitions."""

    def __init__(self, DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=1, shard=0, nshards=1):
        from oracle import oracle as O
        self.o = O.SimpleBatchPianoPIR(DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=seed)
        self.db = np.asarray(rawDB).reshape(DBSize, -1)
        P = BatchSize // 2
        self.PS = (DBSize + P - 1) // P
        self.shard, self.nshards = shard, nshards

    def Preprocessing(self):
        self.o.Preprocessing()

    def QueryWithMask(self, idx):
        idx = np.asarray(idx, dtype=np.uint64)
        rows, _ = self.o.Query(idx)
        rows = rows.copy()
        mine = (idx // self.PS) % self.nshards == self.shard
        rows[~mine] = 0
        ok = mine & rows.any(axis=1) & (rows == self.db[idx.astype(np.int64)]).all(axis=1)
        return rows, ok


def batches():
    rng = np.random.default_rng(7)
    for _ in range(12):
        q = rng.integers(0, N, size=3 * B, dtype=np.uint64)
        q[5] = q[2]
        yield q


def _rank(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pacmann_amd.shard import ShardedBatchPIR
        db = np.random.default_rng(3).integers(0, 2**64, size=N * E, dtype=np.uint64)
        pir = ShardedBatchPIR(N, E * 8, B, db, F, seed=SEED, engine=OracleShard)
        assert (pir.rank, pir.world) == (rank, world)
        pir.Preprocessing()
        res = [pir.QueryWithMask(q) for q in batches()]
        np.save(os.path.join(out_dir, f"rows{rank}.npy"), np.stack([r for r, _ in res]))
        np.save(os.path.join(out_dir, f"ok{rank}.npy"), np.stack([k for _, k in res]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_sharded_batch_pir_world2(oracle):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(2, _free_port(), d), nprocs=2, join=True)
        rows = [np.load(os.path.join(d, f"rows{r}.npy")) for r in range(2)]
        oks = [np.load(os.path.join(d, f"ok{r}.npy")) for r in range(2)]
    assert np.array_equal(rows[0], rows[1]) and np.array_equal(oks[0], oks[1])   # every rank has the answer
    db = np.random.default_rng(3).integers(0, 2**64, size=N * E, dtype=np.uint64)
    ref = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, F, seed=SEED)
    ref.Preprocessing()
    for i, q in enumerate(batches()):
        want, _ = ref.Query(q)
        assert np.array_equal(rows[0][i], want), i
        good = db.reshape(N, E)[q.astype(np.int64)]
        assert np.array_equal(rows[0][i][oks[0][i]], good[oks[0][i]]), i


class SynthShard:
    """A shard over the device-generated DB spec (pm_batchpir_create_synth),
    answered on the host from pacmann_amd.synth_rows: the engine interface the
    bench's BIGANN blocks drive through ShardedBatchPIR."""

    def __init__(self, DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=1, shard=0, nshards=1,
                 db_seed=None):
        assert rawDB is None and db_seed is not None
        self.E, self.db_seed = DBEntryByteNum // 8, db_seed
        self.PS = (DBSize + BatchSize // 2 - 1) // (BatchSize // 2)
        self.shard, self.nshards = shard, nshards

    def QueryWithMask(self, idx):
        from pacmann_amd import synth_rows
        idx = np.asarray(idx, dtype=np.uint64)
        mine = (idx // np.uint64(self.PS)) % np.uint64(self.nshards) == np.uint64(self.shard)
        rows = synth_rows(self.db_seed, idx, self.E)
        rows[~mine] = 0
        return rows, mine


def _rank_synth(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pacmann_amd.shard import ShardedBatchPIR
        pir = ShardedBatchPIR(10**8, 640, 32, None, 8, seed=3, engine=SynthShard, db_seed=41)
        q = np.random.default_rng(5).integers(0, 10**8, size=96).astype(np.uint64)
        rows, ok = pir.QueryWithMask(q)
        np.save(os.path.join(out_dir, f"s{rank}.npy"), rows)
        np.save(os.path.join(out_dir, f"k{rank}.npy"), ok)
    finally:
        dist.destroy_process_group()


def test_sharded_synth_world2():
    """BIGANN-shaped combine (the bench's configs[3] path): two ranks, each
    holding half of the 16 partitions of a 10^8-entry synthetic DB; after the
    all-reduce both hold every row, equal to synth_rows."""
    from pacmann_amd import synth_rows
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank_synth, args=(2, _free_port(), d), nprocs=2, join=True)
        rows = [np.load(os.path.join(d, f"s{r}.npy")) for r in range(2)]
        oks = [np.load(os.path.join(d, f"k{r}.npy")) for r in range(2)]
    q = np.random.default_rng(5).integers(0, 10**8, size=96).astype(np.uint64)
    assert oks[0].all() and oks[1].all()
    assert np.array_equal(rows[0], rows[1])
    assert np.array_equal(rows[0], synth_rows(41, q, 80))
