"""Private graph search over a SHARDED graph DB (VERDICT r02 row ‡; SURVEY.md
§8e): PIRGraphInfo (private-search.go:336-531) fetching every vertex through
the batch PIR whose partitions (batch-pir.go:62-85) are dealt over the ranks,
S sessions per lock-step team, one combine of the team's per-id records per
shared step (pm_search_loop_sharded + pacmann_amd.shard.RecordCombiner).

* world 2 over gloo: two processes on cuda:0 (one GPU per box), each holding
  half of the partitions; both ranks' answers must be identical and equal to
  unsharded oracle runs of the same sessions (same seeds and queries), with
  the same counters, through several maintenance windows.
* world 1 over nccl (RCCL): the same loop with the in-place RCCL all-reduce
  on the team streams (the multi-GPU bench's path with the one rank a box
  allows).
* the synthetic graph (the reference's -input synthetic mode, generated on the
  device from a seed) against the oracle on the same rows materialised on the
  host, and its modelled-peer form (a wider shard layout on one GPU).
"""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, DIM, M, K = 100_000, 128, 32, 10
S, Q, NG = 4, 12, 2
SEEDS = [(700 + i, 800 + i) for i in range(S)]


def _data():
    from pacmann_amd.synth import random_graph, sift_like_vectors
    v = sift_like_vectors(N, DIM, seed=31)
    g = random_graph(N, M, seed=32)
    rng = np.random.default_rng(33)
    qs = np.clip(np.rint(v[rng.integers(0, N, S * Q)] + rng.normal(0, 8, (S * Q, DIM))), 0, 255)
    return v, g, qs.astype(np.float32).reshape(S, Q, DIM)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir, backend, fault=None):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fault and rank == fault[0]:   # this rank's team 0 fails at shared step fault[1] (pm_engine.cpp fault seam)
        os.environ["PM_FAULT_ROUND"] = str(fault[1])
    if backend == "nccl":
        torch.cuda.set_device(0)
    # "native": gloo carries the ncclUniqueIds, the records go through the
    # library's own RCCL communicators (pm_rccl_combine)
    dist.init_process_group("gloo" if backend == "native" else backend, rank=rank, world_size=world)
    try:
        import pacmann_amd as pm
        from pacmann_amd.shard import RcclCombiner, RecordCombiner
        v, g, qs = _data()
        base = pm.PIRGraphInfo.Shard(v, g, rank, world, pir_seed=SEEDS[0][0], search_seed=SEEDS[0][1],
                                     ctx=pm.Context(0))
        base.Preprocess()
        sess = [base] + [base.Session(p, s_, pm.Context(0)) for p, s_ in SEEDS[1:]]
        for x in sess[1:]:
            x.Preprocess()
        comb = RcclCombiner(device=0) if backend == "native" else RecordCombiner(device=0)
        for x in sess:
            x.ctx.timing_reset()
        try:
            ans, wall, on, mt = pm.search_loop_sharded(sess, qs, K, 20, 3, NG, 4, combiner=comb)
        except RuntimeError as e:
            with open(os.path.join(out_dir, f"err{rank}.txt"), "w") as fh:
                fh.write(str(e))
            return
        ncomb = sum(x.ctx.timing_get("host_combine")[0] for x in sess)
        assert ncomb == Q * 20 * NG, ncomb   # one combine per shared step of each team
        if backend != "native":
            assert comb.calls == ncomb, comb.calls
        st = np.array([[*x.counts(), *(x.PIR.stats()[k] for k in ("FinishedBatchNum", "QueriesMadeInPartition",
                                                                  "PrepCount"))] for x in sess])
        np.save(os.path.join(out_dir, f"ans{rank}.npy"), ans)
        np.save(os.path.join(out_dir, f"st{rank}.npy"), st)
    finally:
        if backend == "native" and "comb" in locals():
            comb.close()
        dist.destroy_process_group()


def _oracle_runs(oracle, v, g, qs):
    out = []
    for i, (p, s_) in enumerate(SEEDS):
        o = oracle.Graph(v, g, pir_seed=p, search_seed=s_)
        o.Preprocess()
        a, _, _ = o.SearchLoop(qs[i], K, 20, 3)
        ps = o.pir().stats()
        out.append((a, [*o.counts(), ps["FinishedBatchNum"], ps["QueriesMadeInPartition"], ps["PrepCount"]]))
        del o
    return out


def _run(world, backend, oracle):
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(world, _free_port(), d, backend), nprocs=world, join=True)
        for r in range(world):   # a rank whose loop raised left its message instead of its answers
            e = os.path.join(d, f"err{r}.txt")
            if os.path.exists(e):
                pytest.fail(f"rank {r}: {open(e).read()}")
        ans = [np.load(os.path.join(d, f"ans{r}.npy")) for r in range(world)]
        st = [np.load(os.path.join(d, f"st{r}.npy")) for r in range(world)]
    for r in range(1, world):   # every rank continued the identical searches
        assert np.array_equal(ans[r], ans[0]) and np.array_equal(st[r], st[0])
    v, g, qs = _data()
    for i, (oa, ost) in enumerate(_oracle_runs(oracle, v, g, qs)):
        bad = np.where((ans[0][i] != oa).any(axis=1))[0]
        assert len(bad) == 0, (i, bad[:5].tolist())
        assert st[0][i].tolist() == ost, (i, st[0][i].tolist(), ost)
        assert ost[4] >= 2, i   # every session went through maintenance


def test_sharded_search_gloo_world2(oracle):
    _run(2, "gloo", oracle)


def test_sharded_search_rccl_world1(oracle):
    _run(1, "nccl", oracle)


def test_sharded_search_native_rccl_world1(oracle):
    """The library-native combine (pm_rccl_combine on communicators created
    inside libpacmann.so, no Python on the step path) equals the oracle."""
    _run(1, "native", oracle)


def test_sharded_search_rank_failure_gloo_world2():
    """A failure on one rank mid-search (team 0 of rank 1 at its 7th shared
    step, through the PM_FAULT_ROUND seam) ends the loop on BOTH ranks with an
    error instead of leaving rank 0 inside a collective: the failed rank takes
    its team's next combine turn with the error word set, every rank reads the
    nonzero sum and stops that team, and the other team stops at its next
    turn (pm_engine.cpp group_exchange)."""
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_rank, args=(2, _free_port(), d, "gloo", (1, 7)), nprocs=2, join=True)
        errs = {}
        for r in range(2):
            f = os.path.join(d, f"err{r}.txt")
            assert os.path.exists(f), f"rank {r} finished without an error"
            errs[r] = open(f).read()
    assert "injected" in errs[1], errs
    assert "rank(s) failed" in errs[0], errs


def _synth_materialised(n, dim, m, seed):
    import pacmann_amd as pm
    return pm.graph_synth_rows(n, dim, m, seed, np.arange(n, dtype=np.uint64))


def test_synthetic_graph_search_vs_oracle(ctx, oracle):
    """The device-generated synthetic graph DB (one shard = all partitions):
    sessions through pm_search_loop_sharded without a combine equal oracle
    runs over the same rows materialised on the host."""
    import pacmann_amd as pm
    n, dim, m, seed = 60_000, 64, 32, 77
    base = pm.PIRGraphInfo.Synthetic(n, dim, m, seed, pir_seed=SEEDS[0][0], search_seed=SEEDS[0][1], ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(p, s_) for p, s_ in SEEDS[1:]]
    for x in sess[1:]:
        x.Preprocess()
    v, g = _synth_materialised(n, dim, m, seed)
    rng = np.random.default_rng(5)
    qs = rng.random((S, Q, dim), dtype=np.float32)
    ans, _, _, _ = pm.search_loop_sharded(sess, qs, K, 20, 3, NG, 4)
    for i, (oa, ost) in enumerate(_oracle_runs(oracle, v, g, qs)):
        assert np.array_equal(ans[i], oa), i
        ps = sess[i].PIR.stats()
        assert [*sess[i].counts(), ps["FinishedBatchNum"], ps["QueriesMadeInPartition"], ps["PrepCount"]] == ost, i


def test_synthetic_graph_model_peers(ctx, oracle):
    """Shard 0 of a 2-shard layout with the other shard's partitions answered
    from the graph's spec on the device (model_peers, the bench's way of
    serving a layout wider than the job): the searches match unsharded oracle
    runs except where the oracle's own sub-queries on the other shard's
    partitions failed (no hint hit, ~2^-8 per query) — modelled peers always
    answer."""
    import pacmann_amd as pm
    n, dim, m, seed = 60_000, 64, 32, 78
    base = pm.PIRGraphInfo.Synthetic(n, dim, m, seed, shard=0, nshards=2, pir_seed=SEEDS[0][0],
                                     search_seed=SEEDS[0][1], ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(p, s_) for p, s_ in SEEDS[1:]]
    for x in sess[1:]:
        x.Preprocess()
    v, g = _synth_materialised(n, dim, m, seed)
    rng = np.random.default_rng(6)
    qs = rng.random((S, Q, dim), dtype=np.float32)
    ans, _, _, _ = pm.search_loop_sharded(sess, qs, K, 20, 3, NG, 4, model_peers=True)
    same = total = 0
    for i, (oa, ost) in enumerate(_oracle_runs(oracle, v, g, qs)):
        same += int((ans[i] == oa).all(axis=1).sum())
        total += Q
        assert sess[i].counts()[0] == ost[0], i   # ids fetched: same rounds
    assert same >= 0.75 * total, (same, total)


def test_sharded_loop_odd_entry_layout(ctx, oracle):
    """The records at an entry layout whose neighbour list starts mid-word
    (d = 99, m = 31: 4*d = 396 B, so the list begins 4 B into word 49, and
    E = 65 words with xorSlices' len & ~3 rule zeroing word 64 of every
    answer, as the reference does): the sharded loop over one shard holding
    every partition, two teams, equals unsharded oracle runs answer for answer
    with equal counters."""
    import pacmann_amd as pm
    from pacmann_amd.synth import random_graph
    n, dim, m = 30_000, 99, 31
    rng = np.random.default_rng(41)
    v = rng.random((n, dim), dtype=np.float32)
    g = random_graph(n, m, seed=42)
    base = pm.PIRGraphInfo.Shard(v, g, 0, 1, pir_seed=SEEDS[0][0], search_seed=SEEDS[0][1], ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(p, s_) for p, s_ in SEEDS[1:]]
    for x in sess[1:]:
        x.Preprocess()
    qs = rng.random((S, Q, dim), dtype=np.float32)
    ans, _, _, _ = pm.search_loop_sharded(sess, qs, K, 20, 3, NG, 4)
    for i, (oa, ost) in enumerate(_oracle_runs(oracle, v, g, qs)):
        assert np.array_equal(ans[i], oa), i
        ps = sess[i].PIR.stats()
        assert [*sess[i].counts(), ps["FinishedBatchNum"], ps["QueriesMadeInPartition"], ps["PrepCount"]] == ost, i
