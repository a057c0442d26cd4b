"""Partition-sharded batch PIR over one process per GPU.

SimpleBatchPianoPIR is 16 independent sub-PIRs (batch-pir.go:62-85). Rank r
of a `world`-rank process group holds the partitions p with p % world == r
(their DB slice, keys and hint tables: pm_batchpir_create_shard). Every rank is
fed the same id batches and makes the same bucketing, dummy, drop and
re-preprocessing decisions. It answers its own partitions and leaves the other
entries zero, so one all-reduce SUM of the responses gives every rank the
unsharded answer, bit for bit: the path's only exchange. RCCL has no XOR
reduction, but at most one rank contributes a non-zero entry per id, so the
integer sum equals the XOR (and the per-id success flags, one word per row,
sum to 0 or 1).

The combine is device-resident: each rank's engine writes its responses, with
the success flag as an extra word per row, straight into one device tensor
(pm_batchpir_query_dev copies them HBM to HBM from the partitions' local
caches); under nccl (RCCL over xGMI) that tensor is all-reduced in place and
crosses PCIe to the host once, after the collective.  Under gloo the same
device rows are copied to the host for the CPU collective.

Preprocessing needs no exchange: each rank folds only its own partitions, so
its wall time drops with the rank count.
"""
from __future__ import annotations

import os

import numpy as np


class ShardedBatchPIR:
    """The SimpleBatchPianoPIR surface over a torch.distributed group.

    `engine` builds this rank's shard; by default the GPU engine
    (pacmann_amd.SimpleBatchPianoPIR(..., shard=rank, nshards=world)) on this
    rank's device: `device` if given, else LOCAL_RANK (one process per GPU),
    else the current CUDA device.  A host engine (e.g. the oracle's, in CPU
    tests) has no device path: its responses are combined on the host."""

    def __init__(self, DBSize: int, DBEntryByteNum: int, BatchSize: int, rawDB, FailureProbLog2: int,
                 seed: int = 1, group=None, engine=None, ctx=None, db_seed: int | None = None,
                 device: int | None = None):
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.E = DBEntryByteNum // 8
        self.nccl = dist.get_backend(group) == "nccl"
        gpu_engine = engine is None
        if gpu_engine:
            from . import Context, SimpleBatchPianoPIR
            engine = SimpleBatchPianoPIR
            if ctx is None:
                if device is None:
                    device = int(os.environ.get("LOCAL_RANK", "-1"))
                if device < 0:
                    import torch
                    device = torch.cuda.current_device()
                ctx = Context(device)
        if ctx is not None and device is None:
            device = getattr(ctx, "device", None)
        if self.nccl and not gpu_engine:
            raise ValueError("the nccl combine needs the GPU engine (device-resident responses)")
        kw = {"ctx": ctx} if ctx is not None else {}
        if db_seed is not None:
            kw["db_seed"] = db_seed
        self.pir = engine(DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=seed,
                          shard=self.rank, nshards=self.world, **kw)
        self.device = device
        self.device_path = gpu_engine and hasattr(self.pir, "QueryDevice")
        if self.device_path:
            from . import hip_runtimes
            if len(hip_runtimes()) > 1:
                raise RuntimeError("two HIP runtimes are mapped (libpacmann.so was loaded before torch): "
                                   "import torch before creating any pacmann_amd context")

    def Preprocessing(self):
        self.pir.Preprocessing()

    def DummyPreprocessing(self):
        self.pir.DummyPreprocessing()

    def QueryDevice(self, idx):
        """The combined responses as a fresh device tensor [len(idx), E + 1]
        (int64 view of the uint64 words; column E = success flag), every rank
        holding the same values after the in-place all-reduce.  The tensor
        comes from torch's caching allocator on the current stream, and the
        engine's writes into it wait for that stream's earlier work
        (pm_batchpir_query_dev), so a caller may keep using earlier results."""
        import torch
        ids = np.ascontiguousarray(idx, dtype=np.uint64).ravel()
        with torch.cuda.device(self.device):
            rows = torch.empty((len(ids), self.E + 1), dtype=torch.int64, device=f"cuda:{self.device}")
            stream = torch.cuda.current_stream()
            self.pir.QueryDevice(ids, rows.data_ptr(), stream.cuda_stream)
            if self.nccl:
                self._dist.all_reduce(rows, op=self._dist.ReduceOp.SUM, group=self.group)
            else:   # gloo: the CPU collective over the device rows copied once
                host = rows.cpu()
                self._dist.all_reduce(host, op=self._dist.ReduceOp.SUM, group=self.group)
                rows.copy_(host)
        return rows

    def QueryWithMask(self, idx):
        ids = np.ascontiguousarray(idx, dtype=np.uint64).ravel()
        if self.device_path:
            rows = self.QueryDevice(ids).cpu().numpy().view(np.uint64)   # the one D2H copy
            return np.ascontiguousarray(rows[:, :self.E]), rows[:, self.E].astype(bool)
        import torch   # host engine: combine on the host
        out, ok = self.pir.QueryWithMask(ids)
        rows = torch.from_numpy(np.ascontiguousarray(out).view(np.int64).copy())
        mask = torch.from_numpy(ok.astype(np.int64))
        self._dist.all_reduce(rows, op=self._dist.ReduceOp.SUM, group=self.group)
        self._dist.all_reduce(mask, op=self._dist.ReduceOp.SUM, group=self.group)
        return rows.numpy().view(np.uint64), mask.numpy().astype(bool)

    def Query(self, idx):
        out, _ = self.QueryWithMask(idx)
        return out, None

    def stats(self) -> dict:
        return self.pir.stats()


class RecordCombiner:
    """The combine of pm_search_loop_sharded (private graph search over the
    sharded DB) over a torch.distributed group.

    Each lock-step team of the loop owns one device tensor of int64 words (its
    sessions' per-id records: neighbour words, {dist, ok}), allocated here and
    handed to the library.  After every shared step the library calls back
    with the team index and the HIP stream the records were written on; the
    callback sums the tensor over the group IN PLACE, ordered on that stream:
    nccl (RCCL over xGMI) reduces on the device with the stream made current
    (torch's ProcessGroupNCCL waits for it and makes it wait for the
    collective: no host synchronisation); gloo copies to the host, reduces
    and copies back.  Exactly one rank contributes a non-zero record per id,
    so the integer sum is the unsharded answer.  The library issues the
    callbacks of all teams in one (round, team) order on every rank, so the
    collectives match across ranks."""

    def __init__(self, group=None, device: int | None = None):
        import torch
        import torch.distributed as dist
        self._dist, self._torch = dist, torch
        self.group = group
        self.nccl = dist.get_backend(group) == "nccl"
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "-1"))
            if device < 0:
                device = torch.cuda.current_device()
        self.device = device
        self.bufs = []
        self.error = None
        self.calls = 0

    def prepare(self, words_per_team):
        """Allocate the teams' record tensors; returns their device addresses."""
        torch = self._torch
        self.bufs = [torch.zeros(max(1, int(w)), dtype=torch.int64, device=f"cuda:{self.device}")
                     for w in words_per_team]
        torch.cuda.synchronize(self.device)
        self.error = None
        return [b.data_ptr() for b in self.bufs]

    def callback(self, user, team, ptr, nwords, stream):
        """pm_combine_fn: returns 0, or 1 after recording the exception."""
        torch, dist = self._torch, self._dist
        try:
            t = self.bufs[team]
            if ptr != t.data_ptr() or nwords > t.numel():
                raise RuntimeError(f"team {team}: unexpected record buffer")
            view = t[:nwords]
            with torch.cuda.device(self.device):
                ext = torch.cuda.ExternalStream(stream, device=torch.device("cuda", self.device))
                with torch.cuda.stream(ext):
                    if self.nccl:
                        dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group)
                    else:
                        host = view.cpu()   # on the records' stream: after they are written
                        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
                        view.copy_(host)
            self.calls += 1
            return 0
        except Exception as e:   # the library fails the loop with this status
            self.error = e
            return 1

    def finish(self):
        self._torch.cuda.synchronize(self.device)
        if self.error is not None:
            raise self.error


class RcclUnavailable(RuntimeError):
    """The library-native RCCL combine could not be set up on every rank; the
    ranks agreed on it, so each may fall back to another combine."""


def agree(ok: bool, group=None) -> bool:
    """True iff every rank of `group` passed ok=True (a MIN of the ranks'
    flags over a host collective: gloo, or whatever the group's backend is)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t.item()) == 1


def agreed_setup(setup, teardown=None, group=None):
    """Run setup() on every rank and agree on the outcome: returns setup()'s
    result when every rank succeeded; otherwise every rank tears its own
    result down (teardown(result), if it got one) and raises RcclUnavailable
    with its own error or "another rank failed".  setup() must be bounded
    (pm_rccl_create / pm_rccl_probe are: PM_ETIMEDOUT), so every rank reaches
    the agreement even when a peer never joins the collective part."""
    res, err = None, None
    try:
        res = setup()
    except Exception as e:   # recorded; the agreement decides for every rank alike
        err = e
    if agree(err is None, group):
        return res
    if res is not None and teardown is not None:
        try:
            teardown(res)
        except Exception:
            pass
    raise RcclUnavailable(f"{type(err).__name__}: {err}" if err is not None else "another rank failed its setup")


class RcclCombiner:
    """The library-native combine of pm_search_loop_sharded: RCCL
    communicators over xGMI inside libpacmann.so (pm_rccl_create), one per
    lock-step team, and the C entry point pm_rccl_combine as the loop's
    pm_combine_fn, so no Python and no GIL sit on the per-step path (the
    RecordCombiner's callback is the alternative through torch.distributed).

    `group`: any torch.distributed group of the ranks (gloo is enough): it
    carries rank 0's ncclUniqueIds to the others, once per team count, and the
    agreement.  prepare() is bounded and agreed: the communicators' creation
    (nonblocking, polled) and a 1-word probe all-reduce per team each finish
    within pm_set_option("rccl_timeout_s") seconds, then the ranks take a MIN of
    their success flags; unless every rank succeeded, every rank drops its
    communicators and raises RcclUnavailable (the caller falls back to
    RecordCombiner).  The records live in the library's own device buffers."""

    native = True

    def __init__(self, group=None, device: int | None = None):
        import torch.distributed as dist
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0"))
        self.device = device
        self.h = None
        self.nteams = 0

    def prepare(self, words_per_team):
        """Communicators for len(words_per_team) teams (created collectively on
        first use or when the team count changes); returns the pm_rccl handle
        or raises RcclUnavailable on every rank alike."""
        import ctypes as C

        import torch

        from . import RCCL_ID_BYTES, _check, lib
        n = len(words_per_team)
        if self.h is not None and self.nteams == n:
            return self.h
        self.close()
        # word 0: rank 0 could make the ids (1) or not (0); the ids follow
        buf = np.zeros(8 + n * RCCL_ID_BYTES, dtype=np.uint8)
        err0 = None
        if self.rank == 0:
            try:
                for t in range(n):
                    _check(lib().pm_rccl_unique_id(buf[8 + t * RCCL_ID_BYTES:].ctypes.data_as(C.POINTER(C.c_uint8))))
                buf[0] = 1
            except Exception as e:
                err0 = e
        t_ids = torch.from_numpy(buf.view(np.int64).copy())
        self._dist.broadcast(t_ids, src=self._dist.get_global_rank(self.group, 0) if self.group else 0,
                             group=self.group)
        buf = t_ids.numpy().view(np.uint8).copy()

        def setup():
            if buf[0] != 1:
                raise RcclUnavailable(f"rank 0 could not make RCCL ids: {err0}" if err0 else
                                      "rank 0 could not make RCCL ids")
            h = C.c_void_p()
            _check(lib().pm_rccl_create(self.device, self.world, self.rank,
                                        buf[8:].ctypes.data_as(C.POINTER(C.c_uint8)), n, C.byref(h)))
            try:
                _check(lib().pm_rccl_probe(h))   # one 1-word all-reduce per team, bounded
            except Exception:
                lib().pm_rccl_destroy(h)
                raise
            return h
        self.h = agreed_setup(setup, lambda h: lib().pm_rccl_destroy(h), self.group)
        self.nteams = n
        return self.h

    def finish(self):
        pass

    def close(self):
        if self.h is not None:
            from . import lib
            lib().pm_rccl_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def combiner_with_fallback(words_per_team, device: int, prefer: str = "native", nccl_group_fn=None,
                           gloo_group=None):
    """The sharded loop's combine, agreed by every rank and never left half-set-up:
    the library-native RCCL communicators (RcclCombiner, bounded and probed);
    unless every rank got them, a torch.distributed RCCL group from
    nccl_group_fn() (which must itself probe and agree, returning None on
    failure); else the gloo group through the host.  Returns (combiner, path,
    note) with path "native" | "torch-rccl" | "gloo" and note the reason for a
    fallback (None when the preferred path was taken)."""
    note = None
    if prefer == "native":
        c = RcclCombiner(group=gloo_group, device=device)
        try:
            c.prepare(words_per_team)
            return c, "native", None
        except RcclUnavailable as e:
            note = f"native RCCL combine unavailable ({e}); fell back"
    if prefer in ("native", "torch-rccl") and nccl_group_fn is not None:
        g = nccl_group_fn()
        if g is not None:
            return RecordCombiner(group=g, device=device), "torch-rccl", note
        note = (note + "; " if note else "") + "torch RCCL group unavailable; fell back to gloo"
    return RecordCombiner(group=gloo_group, device=device), "gloo", note
