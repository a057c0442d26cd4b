"""Partition-sharded batch PIR over one process per GPU.

SimpleBatchPianoPIR is 16 independent sub-PIRs (batch-pir.go:62-85). Rank r
of a `world`-rank process group holds the partitions p with p % world == r
(their DB slice, keys and hint tables: pm_batchpir_create_shard). Every rank is
fed the same id batches and makes the same bucketing, dummy, drop and
re-preprocessing decisions. It answers its own partitions and leaves the other
entries zero, so one all-reduce SUM of the entries (and MAX of the success
mask) gives every rank the unsharded answer, bit for bit. This is the path's
only exchange. RCCL has no XOR reduction, but at most one rank contributes a
non-zero entry per id, so an integer sum is exact.

Preprocessing needs no exchange: each rank folds only its own partitions, so
its wall time drops with the rank count.
"""
from __future__ import annotations

import numpy as np


class ShardedBatchPIR:
    """The SimpleBatchPianoPIR surface over a torch.distributed group.

    `engine` builds this rank's shard; by default the GPU engine
    (pacmann_amd.SimpleBatchPianoPIR(..., shard=rank, nshards=world)). The
    combine runs on the group's backend: host tensors for gloo, device tensors
    for nccl (RCCL)."""

    def __init__(self, DBSize: int, DBEntryByteNum: int, BatchSize: int, rawDB, FailureProbLog2: int,
                 seed: int = 1, group=None, engine=None, ctx=None, db_seed: int | None = None,
                 device: int | None = None):
        """db_seed: the shard's rows are generated on its GPU
        (pm_batchpir_create_synth; rawDB None).  device: the CUDA device of the
        combine's tensors under nccl (default: the current one)."""
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.E = DBEntryByteNum // 8
        if engine is None:
            from . import SimpleBatchPianoPIR
            engine = SimpleBatchPianoPIR
        kw = {"ctx": ctx} if ctx is not None else {}
        if db_seed is not None:
            kw["db_seed"] = db_seed
        self.pir = engine(DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=seed,
                          shard=self.rank, nshards=self.world, **kw)
        self._device = "cpu"
        if dist.get_backend(group) == "nccl":
            self._device = "cuda" if device is None else f"cuda:{device}"

    def Preprocessing(self):
        self.pir.Preprocessing()

    def DummyPreprocessing(self):
        self.pir.DummyPreprocessing()

    def QueryWithMask(self, idx):
        import torch
        out, ok = self.pir.QueryWithMask(idx)
        rows = torch.from_numpy(np.ascontiguousarray(out).view(np.int64)).to(self._device)
        mask = torch.from_numpy(ok.astype(np.int32)).to(self._device)
        self._dist.all_reduce(rows, op=self._dist.ReduceOp.SUM, group=self.group)
        self._dist.all_reduce(mask, op=self._dist.ReduceOp.MAX, group=self.group)
        return rows.cpu().numpy().view(np.uint64), mask.cpu().numpy().astype(bool)

    def Query(self, idx):
        out, _ = self.QueryWithMask(idx)
        return out, None

    def stats(self) -> dict:
        return self.pir.stats()
