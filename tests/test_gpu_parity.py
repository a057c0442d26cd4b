"""GPU parity: libpacmann.so (HIP, gfx950) against the CPU oracle, bit-exact.

Every test calls the product through its C ABI (pacmann_amd -> libpacmann.so)
and the restatement through oracle/liboracle.so on identical seeded inputs.
Integer / byte / index results must match bit for bit; the fp32 L2 distances
too (the kernel reproduces l2_distance_amd64.s's accumulation order), so the
tolerance written here is zero ulp.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20240501


def mismatch_report(b, q, got, want, rows, masks=None):
    """Which ids differ and how (zero row / the true row / other)."""
    bad = np.where((got != want).any(axis=1))[0]
    out = [f"batch {b}: {len(bad)} ids differ"]
    for i in bad[:8]:
        g = got[i]
        kind = "zero" if not g.any() else ("db row" if (g == rows[int(q[i])]).all() else "other")
        out.append(f"  pos {i} id {int(q[i])}: got {kind} {int(g[0]):016x}, want {'zero' if not want[i].any() else 'db row' if (want[i] == rows[int(q[i])]).all() else 'other'} {int(want[i][0]):016x}"
                   + (f", masks {[bool(m[i]) for m in masks]}" if masks is not None else ""))
    return "\n".join(out)


def rand_db(n, e, seed=1):
    return np.random.default_rng(seed).integers(0, 2**64, size=n * e, dtype=np.uint64)


# ---------------------------------------------------------------------------
# leaf primitives
# ---------------------------------------------------------------------------
def test_prf_known_answer(ctx):
    import pacmann_amd as pm
    rk = pm.expand_key(bytes(range(16)))
    out = pm.prf_batch(rk, [5], [7], ctx)
    assert int(out[0]) == 0x821E9920390BACED


def test_prf_batch_matches_oracle(ctx, oracle):
    import pacmann_amd as pm
    rng = np.random.default_rng(3)
    for trial in range(4):
        key = rng.bytes(16)
        rk = pm.expand_key(key)
        assert np.array_equal(rk, oracle.expand_key(key))
        n = 200_003
        tags = rng.integers(0, 2**29, size=n, dtype=np.uint64)
        xs = rng.integers(0, 2**35, size=n, dtype=np.uint64)
        assert np.array_equal(pm.prf_batch(rk, tags, xs, ctx), oracle.prf_batch(rk, tags, xs))


@pytest.mark.parametrize("dim", [8, 16, 128, 192, 13, 100, 3])
def test_l2_batch_bitexact(ctx, oracle, dim):
    import pacmann_amd as pm
    rng = np.random.default_rng(dim)
    rows = rng.standard_normal((1000, dim)).astype(np.float32) * 37
    q = rng.standard_normal(dim).astype(np.float32)
    got = pm.l2_batch(q, rows, ctx)
    want = oracle.l2_batch(q, rows)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))   # 0 ulp


def test_l2_msmarco_golden(ctx):
    """Real d=192 vectors from the reference's validation fixture."""
    import pacmann_amd as pm
    from tests.golden_io import load_golden
    g = load_golden("l2_msmarco")
    for qi in range(g["queries"].shape[0]):
        got = pm.l2_batch(g["queries"][qi], g["documents"], ctx)
        assert np.array_equal(got.view(np.uint32), g["dist"][qi].view(np.uint32))


def test_ip_batch(ctx, oracle):
    import pacmann_amd as pm
    rng = np.random.default_rng(5)
    for dim in (128, 192, 7):
        rows = rng.integers(0, 2**32, size=(3001, dim), dtype=np.uint32)
        q = rng.integers(0, 2**32, size=dim, dtype=np.uint32)
        per, s = pm.ip_batch(q, rows, True, ctx)
        want = np.array([oracle.inner_product(r, q) for r in rows], dtype=np.uint32)
        assert np.array_equal(per, want)
        assert s == int(want.astype(np.uint64).sum() % 2**32)
        _, s2 = pm.ip_batch(q, rows, False, ctx)
        assert s2 == s


def ip_closed_form(N, D=128):
    sj = D * (D - 1) // 2
    sj2 = (D - 1) * D * (2 * D - 1) // 6
    return (sj * N * (N - 1) // 2 + sj2 * N) % 2**32


def test_ip_bench_closed_form(ctx, oracle):
    import pacmann_amd as pm
    s, ms = pm.ip_bench(1_000_000, 128, ctx)
    assert s == ip_closed_form(1_000_000)
    assert s == oracle.inner_product_bench(1_000_000, 128, 8)


@pytest.mark.parametrize("ws", [2, 3, 8])
def test_ip_bench_shards(ctx, oracle, ws):
    """The row-sharded scan (pm_ip_bench_shard, bench.py's configs[0] over N
    ranks): each shard's sum equals its closed form and the oracle's scan of
    the same rows, and the shards' sums add up mod 2^32 to the whole fill's."""
    import pacmann_amd as pm
    N, D = 1_000_003, 128
    total = 0
    for r in range(ws):
        r0, r1 = N * r // ws, N * (r + 1) // ws
        s, _ = pm.ip_bench(N, D, ctx, r0=r0, rows=r1 - r0)
        assert s == (ip_closed_form(r1, D) - ip_closed_form(r0, D)) % 2**32, (ws, r)
        if r == ws - 1:   # the last shard's rows materialised: the oracle's InnerProduct over them
            rows = (np.arange(r0, r1, dtype=np.uint32)[:, None] + np.arange(D, dtype=np.uint32)[None, :])
            assert s == oracle.inner_product_scan(rows, np.arange(D, dtype=np.uint32), 1)
        total += s
    assert total % 2**32 == ip_closed_form(N, D)
    assert pm.ip_bench(N, D, ctx, r0=N, rows=0)[0] == 0   # an empty shard
    with pytest.raises(RuntimeError, match="past the fill"):
        pm.ip_bench(N, D, ctx, r0=N - 5, rows=10)


@pytest.mark.slow
def test_ip_bench_full_size(ctx):
    """graphann_test.go:249-283 at N=1e8, D=128 (51.2 GB in HBM)."""
    import pacmann_amd as pm
    s, ms = pm.ip_bench(100_000_000, 128, ctx)
    assert s == 1_178_525_696 == ip_closed_form(100_000_000)


# ---------------------------------------------------------------------------
# PianoPIR
# ---------------------------------------------------------------------------
STATE_KEYS = ["round_keys", "primary_tag", "primary_parity", "primary_pp", "backup_tag",
              "backup_parity", "repl_idx", "repl_val", "hist"]


def assert_state_equal(a, b):
    for k in STATE_KEYS:
        assert np.array_equal(a[k], b[k]), k


# chunk sizes 512 (pipelined fold, SW 4), 1024 (SW 4, 2 loads per thread),
# 2048 (SW 2), 256 (double-buffered fold), odd E (unblocked fold), E < 4 (zero)
@pytest.mark.parametrize("N,E,F", [(18750, 4, 40), (5000, 6, 8), (3000, 5, 8), (2000, 2, 8),
                                   (62500, 80, 8), (262144, 8, 8), (1_000_000, 4, 8)])
def test_pir_preprocessing_state(ctx, oracle, N, E, F):
    import pacmann_amd as pm
    db = rand_db(N, E, seed=N)
    g = pm.PianoPIR(N, E * 8, db, F, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, F, seed=SEED)
    assert g.Config() == o.Config()
    g.Preprocessing()
    o.Preprocessing()
    assert_state_equal(g.export_state(), o.export_state())


@pytest.mark.parametrize("N,E,F", [(18750, 4, 40), (5000, 6, 8), (3000, 5, 8)])
def test_pir_query_sequence(ctx, oracle, N, E, F):
    """TestPIRBasic (pir_test.go:9-58) + bit-exact parity of every response,
    status and the final client state, through one re-preprocessing."""
    import pacmann_amd as pm
    db = rand_db(N, E, seed=7 * N)
    g = pm.PianoPIR(N, E * 8, db, F, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, F, seed=SEED)
    g.Preprocessing()
    o.Preprocessing()
    maxq = g.Config()["MaxQueryNum"]
    rng = np.random.default_rng(N)
    ids = rng.integers(0, N, size=maxq + 40)
    ids[5::17] = ids[3]   # repeats exercise the local cache
    EX = E & ~3
    for i, idx in enumerate(ids):
        real = (i % 13) != 6
        got, err = g.Query(int(idx), real)
        want, st = o.Query(int(idx), real)
        assert (err.code if err else 0) == st, i
        assert np.array_equal(got, want), i
        if real and st == 0:   # property of TestPIRBasic
            assert np.array_equal(got[:EX], db[idx * E: idx * E + EX])
    assert g.Config()["FinishedQueryNum"] == o.Config()["FinishedQueryNum"]
    assert_state_equal(g.export_state(), o.export_state())


def test_pir_server_answer(ctx, oracle):
    import pacmann_amd as pm
    N, E = 40000, 8
    db = rand_db(N, E, 11)
    g = pm.PianoPIR(N, E * 8, db, 8, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, 8, seed=SEED)
    cfg = g.Config()
    rng = np.random.default_rng(1)
    offs = rng.integers(0, cfg["ChunkSize"], size=(37, cfg["SetSize"]), dtype=np.uint32)
    got = g.PrivateQuery(offs)
    for i in range(offs.shape[0]):
        assert np.array_equal(got[i], o.PrivateQuery(offs[i]))


def test_pir_dummy_preprocessing(ctx, oracle):
    import pacmann_amd as pm
    N, E = 9000, 4
    db = rand_db(N, E, 12)
    g = pm.PianoPIR(N, E * 8, db, 8, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, 8, seed=SEED)
    g.DummyPreprocessing()
    o.DummyPreprocessing()
    assert_state_equal(g.export_state(), o.export_state())
    for idx in np.random.default_rng(2).integers(0, N, size=50):
        got, err = g.Query(int(idx), True)
        want, st = o.Query(int(idx), True)
        assert (err.code if err else 0) == st
        assert np.array_equal(got, want)


# ---------------------------------------------------------------------------
# SimpleBatchPianoPIR
# ---------------------------------------------------------------------------
def test_batch_pir_basic(step_ctx, oracle):
    """TestBatchPIRBasic (pir_test.go:60-202) with the GPU path, plus
    bit-exact parity against the oracle for every response."""
    import pacmann_amd as pm
    N, E, B = 1_000_000, 16, 32
    db = np.repeat(np.arange(N, dtype=np.uint64), E)   # rawDB[i*16+j] = i
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 20, seed=SEED, ctx=step_ctx)
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 20, seed=SEED)
    g.Preprocessing()
    o.Preprocessing()
    cfg = g.Config()
    P, PS = cfg["PartitionNum"], cfg["PartitionSize"]
    rng = np.random.default_rng(4)
    # (a) one query per partition
    q1 = np.array([p * PS + rng.integers(0, min(PS, N - p * PS)) for p in range(P)], np.uint64)
    # (b) four per partition
    q2 = np.array([p * PS + rng.integers(0, min(PS, N - p * PS)) for p in range(P) for _ in range(4)],
                  np.uint64)
    for q in (q1, q2):
        got, _ = g.Query(q)
        want, _ = o.Query(q)
        assert np.array_equal(got, want)
        assert np.array_equal(got, db.reshape(N, E)[q])
    # (c) 32 distinct ids all in partition 0: first QueryPerPartition correct, rest zero
    q3 = rng.choice(PS, size=B, replace=False).astype(np.uint64)
    got, _ = g.Query(q3)
    want, _ = o.Query(q3)
    assert np.array_equal(got, want)
    assert np.array_equal(got[:2], db.reshape(N, E)[q3[:2]])
    assert not got[2:].any()


@pytest.mark.parametrize("N,E,B,n", [(200_000, 80, 32, 96), (50_000, 12, 8, 24), (30_000, 6, 32, 200),
                                     (30_000, 6, 4, 2000),
                                     (320_000, 112, 32, 32)])   # configs[2] entry size (896 B), TestBatchPIRPerf batches
def test_batch_pir_sequence(step_ctx, oracle, N, E, B, n):
    """Many batches (duplicates, drops, dummies) through the batch layer's
    re-preprocessing trigger (batch-pir.go:239-245) and, for the last case,
    the per-sub-query FinishedQueryNum == MaxQueryNum path (pir.go:527-530)."""
    import pacmann_amd as pm
    db = rand_db(N, E, N + E)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=step_ctx)
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED)
    g.Preprocessing()
    o.Preprocessing()
    rng = np.random.default_rng(N)
    maxq = g.SubConfig(0)["MaxQueryNum"]
    nb = int(maxq // max(1, n // g.Config()["PartitionNum"])) + 8
    for b in range(min(nb, 400)):
        q = rng.integers(0, N, size=n, dtype=np.uint64)
        q[7::11] = q[1]
        got, _ = g.Query(q)
        want, _ = o.Query(q)
        assert np.array_equal(got, want), b
    sg, so = g.stats(), o.stats()
    for k in ("FinishedBatchNum", "QueriesMadeInPartition", "SupportBatchNum", "PrepCount",
              "LocalStorage", "CommOnline", "CommOffline"):
        assert sg[k] == so[k], k
    for p in range(g.Config()["PartitionNum"]):
        assert_state_equal(g.export_state(p), o.sub(p).export_state())


# ---------------------------------------------------------------------------
# graphann beam search over PIR
# ---------------------------------------------------------------------------
def small_graph(n=4096, d=128, m=32, seed=0):
    from tests.datagen import clustered_vectors, knn_graph
    v = clustered_vectors(n, d, seed=seed)
    return v, knn_graph(v, m)


@pytest.mark.parametrize("nonprivate,bench", [(False, False), (True, False), (False, True)])
def test_search_knn_matches_oracle(ctx, oracle, nonprivate, bench):
    import pacmann_amd as pm
    v, graph = small_graph()
    qs = v[:20] + np.float32(3.0)
    g = pm.PIRGraphInfo(v, graph, nonprivate=nonprivate, skip_prep=bench, pir_seed=5, search_seed=9, ctx=ctx)
    o = oracle.Graph(v, graph, nonprivate=nonprivate, skip_prep=bench, pir_seed=5, search_seed=9)
    g.Preprocess()
    o.Preprocess()
    for q in qs:
        gi, gs = g.SearchKNN(q, 10, 20, 3, bench)
        oi, os_ = o.SearchKNN(q, 10, 20, 3, bench)
        assert np.array_equal(gi, oi)
        assert np.array_equal(gs, os_)
    assert g.counts() == o.counts()


def test_search_loop_with_maintenance(step_ctx, oracle):
    import pacmann_amd as pm
    v, graph = small_graph(n=2048, seed=1)
    qs = v[::37][:30] + np.float32(1.0)
    g = pm.PIRGraphInfo(v, graph, pir_seed=6, search_seed=2, ctx=step_ctx)
    o = oracle.Graph(v, graph, pir_seed=6, search_seed=2)
    g.Preprocess()
    o.Preprocess()
    ga, _, gm = g.SearchLoop(qs, 10, 20, 3)
    oa, _, om = o.SearchLoop(qs, 10, 20, 3)
    assert np.array_equal(ga, oa)
    assert g.PIR.stats()["PrepCount"] == o.pir().stats()["PrepCount"] > 1
    assert g.counts() == o.counts()


@pytest.mark.gpu
def test_batch_query_mask(step_ctx, oracle):
    """pm_batchpir_query_ok: ok => the entry is rawDB[id]; not ok => the id was
    dropped by the bucketing (batch-pir.go:195-200) or failed, entry zero;
    rows identical to the oracle's, across batches with drops and repeats."""
    import pacmann_amd as pm
    N, E, B = 40_000, 8, 16
    db = rand_db(N, E, 99)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=step_ctx)
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED)
    g.Preprocessing()
    o.Preprocessing()
    P = g.Config()["PartitionNum"]
    PS = g.Config()["PartitionSize"]
    rng = np.random.default_rng(5)
    dropped = 0
    for b in range(30):
        q = rng.integers(0, N, size=2 * P, dtype=np.uint64)
        q[:6] = rng.integers(0, PS, size=6)          # crowd partition 0: drops
        q[9] = q[10]                                  # a repeat
        got, ok = g.QueryWithMask(q)
        want, _ = o.Query(q)
        assert np.array_equal(got, want), b
        rows = db.reshape(N, E)[q.astype(np.int64)]
        assert np.array_equal(got[ok], rows[ok]), b
        assert not got[~ok].any(), b
        dropped += int((~ok).sum())
    assert dropped > 0


@pytest.mark.gpu
@pytest.mark.parametrize("nshards", [2, 3])
def test_batch_pir_shards(step_ctx, oracle, nshards):
    """pm_batchpir_create_shard: shards fed the same batches; their entries
    summed (and masks OR-ed) equal the unsharded oracle bit for bit, through
    the batch layer's re-preprocessing trigger; each shard's partitions carry
    the oracle's state; a foreign partition is refused."""
    import pacmann_amd as pm
    N, E, B = 30_000, 6, 8
    db = rand_db(N, E, 77)
    shards = [pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=step_ctx, shard=r, nshards=nshards)
              for r in range(nshards)]
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED)
    for s in shards:
        s.Preprocessing()
    o.Preprocessing()
    P = shards[0].Config()["PartitionNum"]
    rng = np.random.default_rng(11)
    maxq = shards[0].SubConfig(0)["MaxQueryNum"]
    for b in range(int(maxq // 3) + 6):
        q = rng.integers(0, N, size=3 * B, dtype=np.uint64)
        q[4] = q[1]
        parts = [s.QueryWithMask(q) for s in shards]
        got = sum(p[0] for p in parts)
        ok = np.logical_or.reduce([p[1] for p in parts])
        want, _ = o.Query(q)
        if not np.array_equal(got, want):
            state = []
            for p in range(P):
                a, o_ = shards[p % nshards].export_state(p), o.sub(p).export_state()
                for k in STATE_KEYS:
                    if not np.array_equal(a[k], o_[k]):
                        x, y = np.asarray(a[k]).ravel(), np.asarray(o_[k]).ravel()
                        d = np.where(x != y)[0] if x.shape == y.shape else np.array([-1])
                        state.append(f"partition {p} {k}: {len(d)} entries differ, first at {d[:6].tolist()} "
                                     f"(size {x.size})")
            pytest.fail(mismatch_report(b, q, got, want, db.reshape(N, E), [p[1] for p in parts]) + "\n"
                        + "\n".join(state or ["client state equal"]))
        assert not got[~ok].any(), b
    for k in ("FinishedBatchNum", "QueriesMadeInPartition", "SupportBatchNum", "PrepCount"):
        assert all(s.stats()[k] == o.stats()[k] for s in shards), k
    for p in range(P):
        assert_state_equal(shards[p % nshards].export_state(p), o.sub(p).export_state())
    with pytest.raises(Exception):
        shards[0].export_state(1)


# ---------------------------------------------------------------------------
# multi-session serving: several clients over one server DB
# ---------------------------------------------------------------------------
def test_batch_pir_clients_share_server(ctx, oracle):
    """pm_batchpir_create_client: clients with their own keys over one device
    DB answer exactly like independent oracle instances with those keys,
    interleaved batch by batch, through re-preprocessing; destroying the
    server handle first leaves the clients' DB alive."""
    import pacmann_amd as pm
    N, E, B = 30_000, 6, 8
    db = rand_db(N, E, 78)
    srv = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    clients = [srv.Client(SEED + 1 + i) for i in range(2)]
    orc = [oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED + 1 + i) for i in range(2)]
    for c, o in zip(clients, orc):
        c.Preprocessing()
        o.Preprocessing()
    for c in clients:
        c._server = None
    del srv
    rng = np.random.default_rng(12)
    maxq = clients[0].SubConfig(0)["MaxQueryNum"]
    for b in range(int(maxq // 3) + 4):
        for c, o in zip(clients, orc):
            q = rng.integers(0, N, size=3 * B, dtype=np.uint64)
            got, _ = c.Query(q)
            want, _ = o.Query(q)
            if not np.array_equal(got, want):
                pytest.fail(mismatch_report(b, q, got, want, db.reshape(N, E)))
    for c, o in zip(clients, orc):
        assert c.stats()["PrepCount"] == o.stats()["PrepCount"] > 1


def test_search_sessions_concurrent(ctx, oracle):
    """pm_search_loop_sessions: S sessions over one graph and server DB, each
    on its own host thread and stream, give every session the answers, PIR
    counters and maintenance count of an independent oracle run with its seeds."""
    import pacmann_amd as pm
    v, graph = small_graph(n=2048, seed=3)
    base = pm.PIRGraphInfo(v, graph, pir_seed=6, search_seed=2, ctx=ctx)
    base.Preprocess()
    seeds = [(7, 3), (8, 4), (9, 5)]
    sess = [base.Session(p, s) for p, s in seeds]
    for s in sess:
        s.Preprocess()
    rng = np.random.default_rng(4)
    qs = np.stack([v[rng.integers(0, len(v), size=30)] + np.float32(1.0) for _ in seeds])
    ans, wall, on, mt = pm.search_loop_sessions(sess, qs, 10, 20, 3)
    assert wall > 0 and (on > 0).all()
    for i, (p, s) in enumerate(seeds):
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], 10, 20, 3)
        assert np.array_equal(ans[i], oa), i
        assert sess[i].counts() == o.counts(), i
        assert sess[i].PIR.stats()["PrepCount"] == o.pir().stats()["PrepCount"] > 1, i


@pytest.mark.parametrize("ngroups,nthreads", [(1, 0), (1, 2), (2, 3), (3, 4), (5, 2)])
def test_search_sessions_batched(ctx, oracle, ngroups, nthreads):
    """pm_search_loop_batched: five sessions in lock-step, every round of all
    of them one shared step over 5 x 16 partitions; each session's answers,
    PIR counters and maintenance count equal an independent oracle run with
    its seeds (nthreads 2: workers serving several sessions each)."""
    import pacmann_amd as pm
    v, graph = small_graph(n=2048, seed=3)
    base = pm.PIRGraphInfo(v, graph, pir_seed=6, search_seed=2, ctx=ctx)
    base.Preprocess()
    seeds = [(7, 3), (8, 4), (9, 5), (10, 6), (11, 7)]
    sess = [base.Session(p, s) for p, s in seeds]
    for s in sess:
        s.Preprocess()
    rng = np.random.default_rng(5)
    qs = np.stack([v[rng.integers(0, len(v), size=30)] + np.float32(1.0) for _ in seeds])
    ans, wall, on, mt = pm.search_loop_batched(sess, qs, 10, 20, 3, ngroups, nthreads)
    assert wall > 0 and (on > 0).all() and (mt > 0).all()
    for i, (p, s) in enumerate(seeds):
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], 10, 20, 3)
        assert np.array_equal(ans[i], oa), i
        assert sess[i].counts() == o.counts(), i
        assert sess[i].PIR.stats()["PrepCount"] == o.pir().stats()["PrepCount"] > 1, i


@pytest.mark.parametrize("ngroups", [1, 2, 3])
def test_search_device_loop_vs_host_loop(ctx, oracle, ngroups):
    """pm_search_loop_batched's device loop (pm_drl.hip: every round's results,
    GetVertexInfo decode, SearchKNN update / next batch and the batch-PIR
    bucketing on the GPU, chained per team) against the host loop
    (pm_set_option("device_loop", 0)) on fresh sessions with the same seeds,
    and against independent oracle runs: answers, graph counts, batch-PIR
    counters, the id stream's position and the localCache index (a host-path
    batch query after the loop reads it back) all equal.  16,384 vertices
    (PartitionSize 1,024, MaxQueryNum 221): the harness re-preprocesses every
    session after each query, so maintenance runs between the chained queries."""
    import pacmann_amd as pm
    from pacmann_amd.synth import random_graph, sift_like_vectors
    n = 16384
    v = sift_like_vectors(n, 128, seed=71)
    graph = random_graph(n, 32, seed=72)
    seeds = [(80 + i, 90 + i) for i in range(6)]
    rng = np.random.default_rng(73)
    qs = np.stack([np.clip(np.rint(v[rng.integers(0, n, 9)] + rng.normal(0, 8, (9, 128))), 0, 255)
                   .astype(np.float32) for _ in seeds])
    out = {}
    for mode in (1, 0):
        pm.set_option("device_loop", mode)
        try:
            base = pm.PIRGraphInfo(v, graph, pir_seed=1, search_seed=2, ctx=pm.Context(0))
            base.Preprocess()
            sess = [base.Session(p, s) for p, s in seeds]
            for x in sess:
                x.Preprocess()
            for x in sess:
                x.ctx.timing_reset()
            ans, _, _, mt = pm.search_loop_batched(sess, qs, 10, 20, 3, ngroups, 4)
            dev_steps = sum(x.ctx.timing_get("host_dev_steps")[0] for x in sess)
            dev_q = sum(x.ctx.timing_get("host_dev_queries")[1] for x in sess)
            # after the loop, one host-path batch query per session (reads the localCache back)
            probe = np.random.default_rng(74).integers(0, n, size=96).astype(np.uint64)
            extra = [x.PIR.QueryWithMask(probe) for x in sess]
            out[mode] = (ans, [x.counts() for x in sess], [x.PIR.stats() for x in sess], dev_steps, dev_q, extra,
                         (mt > 0).all())
        finally:
            pm.set_option("device_loop", -1)
    (a1, c1, s1, st1, q1, x1, m1), (a0, c0, s0, st0, q0, x0, m0) = out[1], out[0]
    assert st1 == 9 * 20 * ngroups and q1 == 6 * 9, (st1, q1)   # every step of the device run on the GPU loop
    assert st0 == 0
    assert m1 and m0
    assert np.array_equal(a1, a0)
    assert c1 == c0
    for a, b in zip(s1, s0):
        for key in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
            assert a[key] == b[key], key
        assert a["PrepCount"] > 2
    for (ra, oa), (rb, ob) in zip(x1, x0):
        assert np.array_equal(ra, rb) and np.array_equal(oa, ob)
    for i, (p, s) in enumerate(seeds):
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], 10, 20, 3)
        assert np.array_equal(a1[i], oa), i
        assert c1[i] == o.counts(), i


def test_device_loop_fault_marks_sessions_lost(ctx, oracle):
    """A device-loop call that fails after queueing work: the
    sessions' host mirrors (FinishedBatchNum, QueriesMadeInPartition, the
    search streams) were advanced for the queued query while its device state
    (dummy counters, FinishedQueryNum, localCache index, id stream) was never
    read back.  Fault injected before query 1 (query 0 queued and running):
    the call fails with the injected error, the teams' streams are drained,
    and every later call on those sessions fails with "session state lost"
    instead of reissuing dummy-counter values the server has seen.  Fresh
    sessions of the same base still serve and equal the oracle."""
    import pacmann_amd as pm
    from pacmann_amd.synth import random_graph, sift_like_vectors
    n = 16384
    v = sift_like_vectors(n, 128, seed=171)
    graph = random_graph(n, 32, seed=172)
    rng = np.random.default_rng(173)
    qs = np.stack([np.clip(np.rint(v[rng.integers(0, n, 3)] + rng.normal(0, 8, (3, 128))), 0, 255)
                   .astype(np.float32) for _ in range(4)])
    base = pm.PIRGraphInfo(v, graph, pir_seed=1, search_seed=2, ctx=pm.Context(0))
    base.Preprocess()
    pm.set_option("device_loop", 1)
    try:
        sess = [base.Session(180 + i, 190 + i) for i in range(4)]
        for x in sess:
            x.Preprocess()
        pm.set_option("fault_drl_query", 1)
        try:
            with pytest.raises(RuntimeError, match="injected fault"):
                pm.search_loop_batched(sess, qs, 10, 20, 3, 2, 4)
        finally:
            pm.set_option("fault_drl_query", -1)
        with pytest.raises(RuntimeError, match="session state lost"):
            pm.search_loop_batched(sess, qs, 10, 20, 3, 2, 4)
        with pytest.raises(RuntimeError, match="session state lost"):
            pm.search_loop_batched(sess[:1], qs[:1], 10, 20, 3, 1, 1)
        seeds = [(280 + i, 290 + i) for i in range(2)]
        fresh = [base.Session(p, s) for p, s in seeds]
        for x in fresh:
            x.Preprocess()
        ans, _, _, _ = pm.search_loop_batched(fresh, qs[:2], 10, 20, 3, 1, 2)
    finally:
        pm.set_option("device_loop", -1)
    for i, (p, s) in enumerate(seeds):
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], 10, 20, 3)
        assert np.array_equal(ans[i], oa), i


def test_search_sessions_batched_wide_entries(ctx, oracle):
    """Entries wider than the answer kernels' small row buffer: dim 500, m 16
    gives E = (2000 + 64) / 8 = 258 words, which passes k_answer_p's even-E
    and gather-slice tests but not its RowBufT<kSmallE = 256> row.  Twelve
    sessions in one lock-step group (12 x 48 = 576 sub-queries per shared
    step, above k_answer_p's 512 threshold, with pre-expanded query sets) must
    take a kernel whose row holds all 258 words and equal independent oracle
    runs (answers, counts, batch-PIR counters through maintenance)."""
    import pacmann_amd as pm
    from pacmann_amd.synth import random_graph, sift_like_vectors
    n, dim, m = 4096, 500, 16
    v = sift_like_vectors(n, dim, seed=41)
    graph = random_graph(n, m, seed=42)
    base = pm.PIRGraphInfo(v, graph, pir_seed=43, search_seed=44, ctx=ctx)
    base.Preprocess()
    assert base.PIR.Config()["DBEntryByteNum"] == (dim + m) * 4
    seeds = [(50 + i, 60 + i) for i in range(12)]
    sess = [base.Session(p, s) for p, s in seeds]
    for s in sess:
        s.Preprocess()
    rng = np.random.default_rng(45)
    qs = np.stack([np.clip(np.rint(v[rng.integers(0, n, 12)] + rng.normal(0, 8, (12, dim))), 0, 255)
                   .astype(np.float32) for _ in seeds])
    ans, wall, on, mt = pm.search_loop_batched(sess, qs, 10, 20, 3, 1, 4)
    for i, (p, s) in enumerate(seeds):
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], 10, 20, 3)
        assert np.array_equal(ans[i], oa), i
        assert sess[i].counts() == o.counts(), i
        assert sess[i].PIR.stats()["PrepCount"] == o.pir().stats()["PrepCount"] > 1, i


def test_batch_pir_group(ctx, oracle):
    """pm_batchpir_group_query: five clients of one server answered with one
    shared step per call; every client's entries, success flags, counters and
    re-preprocessing equal an independent oracle SimpleBatchPianoPIR with its
    seed, through the batch layer's own re-preprocessing trigger."""
    import pacmann_amd as pm
    N, E, B = 30_000, 8, 8
    db = rand_db(N, E, 91)
    server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    server.Preprocessing()
    seeds = [SEED, 11, 12, 13, 14]
    clients = [server] + [server.Client(sd, pm.Context(0)) for sd in seeds[1:]]
    for c in clients[1:]:
        c.Preprocessing()
    grp = pm.BatchPIRGroup(clients)
    ors = [oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=sd) for sd in seeds]
    for o in ors:
        o.Preprocessing()
    rng = np.random.default_rng(21)
    maxq = server.SubConfig(0)["MaxQueryNum"]
    for b in range(int(maxq // 3) + 6):
        q = rng.integers(0, N, size=(len(clients), 3 * B), dtype=np.uint64)
        q[:, 4] = q[:, 1]
        out, ok = grp.QueryWithMask(q)
        for i, o in enumerate(ors):
            want, _ = o.Query(q[i])
            assert np.array_equal(out[i], want), (b, i)
            rows = db.reshape(N, E)[q[i].astype(np.int64)]
            assert np.array_equal(out[i][ok[i]], rows[ok[i]]), (b, i)
            assert not out[i][~ok[i]].any(), (b, i)
    for c, o in zip(clients, ors):
        for k in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
            assert c.stats()[k] == o.stats()[k], k
        assert c.stats()["PrepCount"] > 1


@pytest.mark.parametrize("opts,path", [
    ({"match_resolve": 0, "match_part": 1, "match_part8": 1}, "part8"),   # k_match_part8 -> k_resolve
    ({"match_resolve": 0, "match_part": 1, "match_part8": 0}, "part"),    # k_match_part (LDS-merged) -> k_resolve
    ({"match_resolve": 0, "match_part": 0}, ""),                           # k_match per (sub-query, block)
], ids=["part8", "part", "per_subquery"])
def test_batch_pir_group_hint_search_paths(ctx, oracle, opts, path):
    """Every hint-search form (pm_set_option) answers a group's batches exactly
    as the oracle: five clients, PH 1,792 (one full and one partial 1,024-hint
    block; PH % 8 == 0 so k_match_part8 applies), repeated ids, through the
    batch layer's re-preprocessing; entries, flags and counters compared.  The
    engine's per-path launch counters (host_path_match*) prove that the forced
    kernel, and only it, ran every step."""
    import pacmann_amd as pm
    N, E, B = 30_000, 8, 8
    db = rand_db(N, E, 93)
    try:
        for k, v in opts.items():
            pm.set_option(k, v)
        server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
        server.Preprocessing()
        assert server.SubConfig(0)["PrimaryHintNum"] == 1792
        seeds = [SEED, 21, 22, 23, 24]
        clients = [server] + [server.Client(sd, pm.Context(0)) for sd in seeds[1:]]
        for c in clients[1:]:
            c.Preprocessing()
        grp = pm.BatchPIRGroup(clients)
        ors = [oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=sd) for sd in seeds]
        for o in ors:
            o.Preprocessing()
        rng = np.random.default_rng(23)
        maxq = server.SubConfig(0)["MaxQueryNum"]
        ctx.timing_reset()
        ctx.timing(2)   # the shared steps run on the first client's context: which kernels ran
        for b in range(int(maxq // 3) + 3):
            q = rng.integers(0, N, size=(len(clients), 3 * B), dtype=np.uint64)
            q[:, 5] = q[:, 2]
            out, ok = grp.QueryWithMask(q)
            for i, o in enumerate(ors):
                want, _ = o.Query(q[i])
                assert np.array_equal(out[i], want), (b, i)
        ctx.sync()
        ctx.timing(False)
        n_match = ctx.timing_get("hint_match")[0]
        assert n_match > 0 and ctx.timing_get("resolve")[0] > 0
        counts = {p: ctx.timing_get("host_path_match" + ("_" + p if p else ""))[0] for p in ("part8", "part", "")}
        assert counts[path] == n_match and sum(counts.values()) == n_match, counts
        for c, o in zip(clients, ors):
            for k in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
                assert c.stats()[k] == o.stats()[k], k
            assert c.stats()["PrepCount"] > 1
    finally:
        ctx.timing(False)
        for k in ("match_part", "match_part8", "match_resolve"):
            pm.set_option(k, -2)


def test_set_option_rejects_unknown():
    import pacmann_amd as pm
    with pytest.raises(RuntimeError, match="unknown option"):
        pm.set_option("no_such_path", 1)


def test_batch_pir_group_rejects(ctx):
    """pm_batchpir_group_create refuses clients of different servers and a
    client listed twice; the ids must hold one row per client."""
    import pacmann_amd as pm
    N, E, B = 4_000, 4, 8
    a = pm.SimpleBatchPianoPIR(N, E * 8, B, rand_db(N, E, 1), 8, seed=1, ctx=ctx)
    b = pm.SimpleBatchPianoPIR(N, E * 8, B, rand_db(N, E, 2), 8, seed=1, ctx=ctx)
    a.Preprocessing()
    b.Preprocessing()
    with pytest.raises(RuntimeError, match="one server"):
        pm.BatchPIRGroup([a, b])
    with pytest.raises(RuntimeError, match="twice"):
        pm.BatchPIRGroup([a, a])
    c = a.Client(5, pm.Context(0))
    c.Preprocessing()
    grp = pm.BatchPIRGroup([a, c])
    with pytest.raises(ValueError):
        grp.QueryWithMask(np.zeros((3, B), dtype=np.uint64))
    out, ok = grp.QueryWithMask(np.arange(2 * B, dtype=np.uint64).reshape(2, B))
    assert out.shape == (2, B, E) and ok.shape == (2, B)


def test_search_sessions_batched_rejects(ctx):
    """pm_search_loop_batched refuses sessions it cannot share a step between:
    clients of different server DBs, a session twice, an unpreprocessed one."""
    import pacmann_amd as pm
    v, graph = small_graph(n=1024, seed=4)
    bases = []
    for seed in (1, 2):
        b = pm.PIRGraphInfo(v, graph, pir_seed=seed, search_seed=seed, ctx=pm.Context(0))
        b.Preprocess()
        bases.append(b)
    a, b = bases[0].Session(3, 3), bases[1].Session(4, 4)
    for s_ in (a, b):
        s_.Preprocess()
    qs = np.stack([v[:2], v[:2]])
    with pytest.raises(RuntimeError):
        pm.search_loop_batched([a, b], qs, 10, 20, 3)
    with pytest.raises(RuntimeError):
        pm.search_loop_batched([a, a], qs, 10, 20, 3)
    c = bases[0].Session(5, 5)   # not preprocessed
    with pytest.raises(RuntimeError):
        pm.search_loop_batched([a, c], qs, 10, 20, 3)


# ---------------------------------------------------------------------------
# graph construction (build_graph.go) and kNN ground truth
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n,dim", [(3000, 128), (1500, 192), (777, 100), (40, 16)])
def test_knn_exact_integer_rows(ctx, oracle, n, dim):
    """pm_knn on integer-valued rows (SIFT's uint8 semantics): ids and L2Dist
    values identical to brute force, incl. duplicate rows (ties -> id order),
    a ragged tail tile and n < 64."""
    import pacmann_amd as pm
    from tests.datagen import clustered_vectors
    v = clustered_vectors(n, dim, seed=n)
    v[5] = v[3]                     # exact duplicates: ties broken by id
    q = np.clip(v[:: max(1, n // 60)][:60] + 1, 0, 255).astype(np.float32)
    k = min(20, n)
    gi, gd = pm.knn(v, q, k, ctx, with_dist=True)
    oi, od = oracle.knn(v, q, k)
    assert np.array_equal(gi, oi)
    assert np.array_equal(gd.view(np.uint32), od.view(np.uint32))


def test_knn_float_rows_overlap(ctx, oracle):
    """General float rows: the bf16 prefilter keeps 64 candidates for the exact
    re-rank of the top 10; the result matches brute force on >= 99% of ids,
    and every returned distance is the exact L2Dist of its id."""
    import pacmann_amd as pm
    rng = np.random.default_rng(3)
    v = rng.standard_normal((4000, 192)).astype(np.float32)
    q = rng.standard_normal((50, 192)).astype(np.float32)
    gi, gd = pm.knn(v, q, 10, ctx, with_dist=True)
    oi, _ = oracle.knn(v, q, 10)
    same = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(gi, oi)])
    assert same >= 0.99, same
    for r in range(5):
        want = oracle.l2_batch(q[r], v[gi[r]])
        assert np.array_equal(gd[r].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("n,dim,m", [(4096, 128, 32), (1200, 192, 32), (500, 100, 16), (40, 16, 32)])
def test_build_graph_matches_oracle(ctx, oracle, n, dim, m):
    """pm_build_graph (GPU kNN + robustPrune, host edge sampling and fill) is
    bit-identical to the oracle's restatement of CreateGraphBasedOnNGT with
    exact candidates; no row lists itself."""
    import pacmann_amd as pm
    from tests.datagen import clustered_vectors
    v = clustered_vectors(n, dim, seed=7 + n)
    g, t = pm.build_graph(v, m, 1.2, seed=9, ctx=ctx)
    o = oracle.build_graph(v, m, 1.2, seed=9)
    if not np.array_equal(g, o):
        bad = np.where((g != o).any(axis=1))[0]
        pytest.fail(f"{len(bad)} rows differ, first {bad[:5].tolist()}: {g[bad[0]].tolist()} vs {o[bad[0]].tolist()}")
    assert (g != np.arange(n, dtype=np.uint32)[:, None]).all()
    assert t["knn_s"] > 0


def test_built_graph_search_parity(ctx, oracle):
    """A private search over the GPU-built graph: same answers as the oracle,
    and recall@10 against pm_knn's ground truth is identical (the ±0.5-point
    recall gate of SURVEY.md §8d, met exactly)."""
    import pacmann_amd as pm
    from pacmann_amd.report import compute_recall
    from tests.datagen import clustered_vectors
    v = clustered_vectors(4096, 128, seed=21)
    g, _ = pm.build_graph(v, 32, 1.2, seed=3, ctx=ctx)
    rng = np.random.default_rng(5)
    qs = np.clip(np.rint(v[rng.integers(0, len(v), 40)] + rng.normal(0, 8, (40, 128))), 0, 255).astype(np.float32)
    gt = pm.knn(v, qs, 10, ctx)
    gi = pm.PIRGraphInfo(v, g, pir_seed=4, search_seed=6, ctx=ctx)
    gi.Preprocess()
    og = oracle.Graph(v, g, pir_seed=4, search_seed=6)
    og.Preprocess()
    ga, _, _ = gi.SearchLoop(qs, 10, 20, 3)
    oa, _, _ = og.SearchLoop(qs, 10, 20, 3)
    assert np.array_equal(ga, oa)
    assert compute_recall(gt, ga, 10) == compute_recall(oracle.knn(v, qs, 10)[0], oa, 10)


# ---------------------------------------------------------------------------
# BIGANN-shaped partitions (BASELINE.json configs[3]/[4]): ChunkSize 8,192 /
# 16,384, SetSize 764 / 1,028, PrimaryHintNum > 8,192.  These take the
# unblocked fold, the three-kernel step and the split gather (k_gather).
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("N,E,nq", [(6_250_000, 12, 400), (16_800_000, 4, 300)])
def test_pir_bigann_partition(ctx, oracle, N, E, nq):
    """One PianoPIR the size of a BIGANN-100M partition (CS 8,192, SS 764) and a
    16,384-chunk one (BIGANN-1B's CS): preprocessing state, every response and
    status (real and dummy queries, repeats through the local cache) and the
    final client state bit-exact against the oracle."""
    import pacmann_amd as pm
    db = rand_db(N, E, seed=N + 1)
    g = pm.PianoPIR(N, E * 8, db, 8, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, 8, seed=SEED)
    cfg = g.Config()
    assert cfg == o.Config() and cfg["ChunkSize"] >= 8192 and cfg["SetSize"] >= 256
    g.Preprocessing()
    o.Preprocessing()
    assert_state_equal(g.export_state(), o.export_state())
    rng = np.random.default_rng(N)
    ids = rng.integers(0, N, size=nq)
    ids[7::23] = ids[2]
    ids[11::37] = ids[5] ^ 1   # neighbours in the same chunk
    EX = E & ~3
    for i, idx in enumerate(ids):
        real = (i % 9) != 4
        got, err = g.Query(int(idx), real)
        want, st = o.Query(int(idx), real)
        assert (err.code if err else 0) == st, i
        assert np.array_equal(got, want), i
        if real and st == 0:
            assert np.array_equal(got[:EX], db[idx * E: idx * E + EX])
    assert_state_equal(g.export_state(), o.export_state())


def test_batch_synth_db_bigann_shard(ctx):
    """BIGANN-100M over 4 GPUs, rank 0's shard (4 partitions, 16 GB generated
    on the device by pm_batchpir_create_synth): pir_test.go's property over
    search-shaped batches of 96 ids — every successful entry equals its DB row
    (recomputed on the host from the synth spec), every other entry is zero,
    and only ids of this shard's partitions succeed."""
    import pacmann_amd as pm
    N, E, ns = 100_000_000, 80, 4
    g = pm.SimpleBatchPianoPIR(N, E * 8, 32, None, 8, seed=SEED, ctx=ctx, shard=0, nshards=ns, db_seed=5)
    g.Preprocessing()
    PS = g.Config()["PartitionSize"]
    rng = np.random.default_rng(9)
    nok = 0
    for b in range(25):
        q = rng.integers(0, N, size=96).astype(np.uint64)
        out, ok = g.QueryWithMask(q)
        mine = (q // np.uint64(PS)) % np.uint64(ns) == 0
        assert not (ok & ~mine).any(), b
        assert np.array_equal(out[ok], pm.synth_rows(5, q[ok], E)), b
        assert not out[~ok].any(), b
        nok += int(ok.sum())
    assert nok > 25 * 96 // ns // 2
    rows = pm.synth_rows(5, [0, 1, N - 1], E)
    assert rows.shape == (3, E) and len({int(r[0]) for r in rows}) == 3


def test_build_graph_hub_list_matches_oracle(ctx, oracle):
    """A hub vertex (the centre of a shell of points in 64-d: every vertex's
    nearest) collects every in-edge, so its sampled connection list is longer
    than the prune kernel's LDS sort (4,096): that list takes the presorted
    path (GPU distances, host sort of the exact keys, the same greedy pass).
    The graph is bit-identical to the oracle's restatement."""
    import pacmann_amd as pm
    rng = np.random.default_rng(31)
    n, d = 8000, 64
    u = rng.standard_normal((n, d))
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    v = np.clip(np.rint(128 + 100 * u), 0, 255).astype(np.float32)
    v[0] = 128   # the hub
    # the hub is in (nearly) every vertex's 1.5m candidates, so robustPrune
    # keeps it first and its bi-directional list holds that many in-edges
    ids, _ = oracle.knn(v, v, 49)
    assert (ids == 0).any(axis=1).sum() > 6000
    g, _ = pm.build_graph(v, 32, 1.2, seed=5, ctx=ctx)
    o = oracle.build_graph(v, 32, 1.2, seed=5)
    if not np.array_equal(g, o):
        bad = np.where((g != o).any(axis=1))[0]
        pytest.fail(f"{len(bad)} rows differ, first {bad[:5].tolist()}")
