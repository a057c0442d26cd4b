"""GPU parity at the benchmark configurations' own shapes (BASELINE.json
configs[1]-[4]), not scaled-down stand-ins.

Each test drives the product through its C ABI at the partition geometry the
bench measures and compares with the oracle on the same seeds, or — where the
oracle cannot hold the data (the 1B-entry shard) — with the reference's own
property (pir_test.go:45-49: a successful answer is the DB row, anything else
is zero), recomputing every row on the host.

  configs[1] SIFT1M:    1e6 x 640 B, 16 partitions (CS 512 / SS 124), search
                        sessions through the batched serving loop
  configs[2] MS-MARCO:  3,201,821 x 896 B, 16 partitions (CS 1,024 / SS 196 /
                        E 112): batch PIR and the d=192 private search
  configs[4] BIGANN-1B: CS 16,384 / SS 3,816 partitions (62.5M entries), one
                        vs the oracle and the 8-way shard 0 at full size

The oracle runs its hint fold on several threads (oracle.set_prep_threads:
the hint space is split, the state is identical), so each test finishes in
well under two minutes on the GPU box's host share.
"""
import numpy as np
import pytest

from tests.test_gpu_parity import SEED, STATE_KEYS, assert_state_equal, mismatch_report, rand_db

pytestmark = pytest.mark.gpu


def state_diff(a, b):
    out = []
    for k in STATE_KEYS:
        x, y = np.asarray(a[k]).ravel(), np.asarray(b[k]).ravel()
        if x.shape != y.shape or not np.array_equal(x, y):
            d = np.where(x != y)[0] if x.shape == y.shape else np.array([-1])
            out.append(f"{k}: {len(d)} entries differ, first at {d[:6].tolist()}")
    return out


# ---------------------------------------------------------------------------
# configs[4]: BIGANN-1B partition geometry (CS 16,384, SS 3,816, PH 114,688)
# ---------------------------------------------------------------------------
def test_pir_bigann_1b_partition_vs_oracle(ctx, oracle):
    """One PianoPIR of a BIGANN-1B partition's size (62.5M entries: CS 16,384,
    SS 3,816 — the k_gather split the 1B shard takes) with 32-B entries:
    preprocessing state, 300 responses and statuses (real and dummy, repeats
    through the local cache, same-chunk neighbours) and the final state equal
    the oracle's."""
    import pacmann_amd as pm
    N, E = 62_500_000, 4
    db = rand_db(N, E, seed=62)
    g = pm.PianoPIR(N, E * 8, db, 8, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, 8, seed=SEED)
    cfg = g.Config()
    assert cfg == o.Config()
    assert (cfg["ChunkSize"], cfg["SetSize"], cfg["PrimaryHintNum"], cfg["MaxQueryPerChunk"]) == (16384, 3816, 114688, 112)
    g.Preprocessing()
    o.Preprocessing()
    diff = state_diff(g.export_state(), o.export_state())
    assert not diff, diff
    rng = np.random.default_rng(N)
    ids = rng.integers(0, N, size=300)
    ids[7::23] = ids[2]
    ids[11::37] = ids[5] ^ 1
    for i, idx in enumerate(ids):
        real = (i % 9) != 4
        got, err = g.Query(int(idx), real)
        want, st = o.Query(int(idx), real)
        assert (err.code if err else 0) == st, i
        assert np.array_equal(got, want), i
        if real and st == 0:
            assert np.array_equal(got, db[idx * E: idx * E + E]), i
    diff = state_diff(g.export_state(), o.export_state())
    assert not diff, diff


def test_batch_bigann_1b_shard_full_size(ctx):
    """configs[4] as the bench lays it out: 1e9 entries of 640 B, partitions
    dealt 8-way, shard 0 = partitions 0 and 8 (2 x 62.5M rows = 80 GB
    generated on the device).  25 search-shaped rounds of 96 ids: every
    successful entry equals its DB row (recomputed on the host from the synth
    spec), every other entry is zero, only shard 0's partitions answer, and
    most of them do."""
    import pacmann_amd as pm
    N, E, ns = 1_000_000_000, 80, 8
    g = pm.SimpleBatchPianoPIR(N, E * 8, 32, None, 8, seed=SEED, ctx=ctx, shard=0, nshards=ns, db_seed=41)
    sc = g.SubConfig(0)
    assert (sc["ChunkSize"], sc["SetSize"]) == (16384, 3816)
    g.Preprocessing()
    PS = g.Config()["PartitionSize"]
    rng = np.random.default_rng(17)
    nok = unexplained = 0
    for b in range(25):
        q = rng.integers(0, N, size=96).astype(np.uint64)
        q[5] = q[3]
        out, ok = g.QueryWithMask(q)
        part = q // np.uint64(PS)
        mine = part % np.uint64(ns) == 0
        assert not (ok & ~mine).any(), b
        assert np.array_equal(out[ok], pm.synth_rows(41, q[ok], E)), b
        assert not out[~ok].any(), b
        nok += int(ok.sum())
        # an id of this shard that failed: its bucket overflowed (queryNumToMake
        # = 96 / 16 = 6 per partition, batch-pir.go:195-200) or, with
        # probability ~2^-8 per query, no hint hit
        crowded = {int(p) for p in part if (part == p).sum() > 6}
        unexplained += sum(1 for i in np.where(mine & ~ok)[0] if int(part[i]) not in crowded)
    assert nok > 0 and unexplained <= 3, (nok, unexplained)


# ---------------------------------------------------------------------------
# configs[2]: MS-MARCO batch PIR, the TestBatchPIRPerf shape at full size
# ---------------------------------------------------------------------------
def test_batch_pir_msmarco_full_vs_oracle(ctx, oracle):
    """3,201,821 entries of 896 B, BatchSize 32 (16 partitions of CS 1,024 /
    SS 196), F = 8: every partition's preprocessing state, then 2,740 batches
    of 32 uniform ids with repeats — past the batch layer's re-preprocessing
    trigger (QueriesMadeInPartition >= MaxQueryNum - 2, batch-pir.go:239-245)
    — every response equal to the oracle's, then the counters and every
    partition's final state."""
    import pacmann_amd as pm
    N, E, B = 3_201_821, 112, 32
    db = rand_db(N, E, seed=77)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED)
    sc = g.SubConfig(0)
    assert (sc["ChunkSize"], sc["SetSize"], sc["MaxQueryNum"]) == (1024, 196, 5460)
    g.Preprocessing()
    o.Preprocessing()
    P = g.Config()["PartitionNum"]
    for p in range(P):
        diff = state_diff(g.export_state(p), o.sub(p).export_state())
        assert not diff, (p, diff)
    rng = np.random.default_rng(78)
    rows = db.reshape(N, E)
    nb = (sc["MaxQueryNum"] - 2) // 2 + 12
    good = 0
    for b in range(nb):
        q = rng.integers(0, N, size=B, dtype=np.uint64)
        if b % 5 == 0:
            q[9] = q[2]
        got, _ = g.Query(q)
        want, _ = o.Query(q)
        if not np.array_equal(got, want):
            pytest.fail(mismatch_report(b, q, got, want, rows))
        good += int((got == rows[q.astype(np.int64)]).all(axis=1).sum())
    assert good > nb * B // 2
    sg, so = g.stats(), o.stats()
    for k in ("FinishedBatchNum", "QueriesMadeInPartition", "SupportBatchNum", "PrepCount"):
        assert sg[k] == so[k], k
    assert sg["PrepCount"] == 2
    for p in range(P):
        diff = state_diff(g.export_state(p), o.sub(p).export_state())
        assert not diff, (p, diff)


def test_batch_pir_group_msmarco_bench_shape(ctx, oracle):
    """The bench's config2 `clients_grouped` shape: 32 clients of the one
    3,201,821 x 896 B server, every round ONE shared step over their 512
    partitions (2 sub-queries each: the grouped hint search k_match_part8,
    k_resolve, k_answer); 40 rounds of 32 uniform ids per client; clients 0,
    9, 20 and 31 compared response for response with independent oracle
    clients of the same seeds, then their counters."""
    import pacmann_amd as pm
    from concurrent.futures import ThreadPoolExecutor
    N, E, B, K = 3_201_821, 112, 32, 32
    db = rand_db(N, E, seed=79)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    g.Preprocessing()
    seeds = [SEED] + [2000 + i for i in range(1, K)]
    clients = [g] + [g.Client(sd, pm.Context(0)) for sd in seeds[1:]]
    for c in clients[1:]:
        c.Preprocessing()
    grp = pm.BatchPIRGroup(clients)
    check = [0, 9, 20, 31]

    def make(i):
        o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=seeds[i])
        o.Preprocessing()
        return i, o
    with ThreadPoolExecutor(max_workers=len(check)) as ex:
        ors = dict(ex.map(make, check))
    rng = np.random.default_rng(80)
    ctx.timing_reset()
    ctx.timing(2)   # the shared steps run on the first client's context
    try:
        for b in range(40):
            q = rng.integers(0, N, size=(K, B), dtype=np.uint64)
            if b % 4 == 0:
                q[:, 7] = q[:, 3]
            out, ok = grp.QueryWithMask(q)
            for i in check:
                want, _ = ors[i].Query(q[i])
                assert np.array_equal(out[i], want), (b, i)
        ctx.sync()
    finally:
        ctx.timing(False)
    assert ctx.timing_get("hint_match")[0] > 0 and ctx.timing_get("answer")[0] > 0
    for i in check:
        sc, so = clients[i].stats(), ors[i].stats()
        for k in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
            assert sc[k] == so[k], (i, k)


# ---------------------------------------------------------------------------
# private search at full size: SIFT1M (configs[1]) and MS-MARCO d=192
# ---------------------------------------------------------------------------
def _sessions_vs_oracle(ctx, oracle, v, graph, qs_per_session, k, seeds, ngroups, nthreads, check=None,
                        oracle_workers=8, timing=False):
    """Serve the sessions through pm_search_loop_batched, then replay each
    checked session (`check`: indices, default all) as an independent oracle
    client with the same seeds and queries.  Answers, counts and batch-PIR
    counters must be equal.  Each oracle client is freed as soon as it has
    been compared (a SIFT1M client holds 0.85 GB, an MS-MARCO one 3.4 GB).
    timing: kernel timings of the shared steps are returned too."""
    import pacmann_amd as pm
    base = pm.PIRGraphInfo(v, graph, pir_seed=seeds[0][0], search_seed=seeds[0][1], ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(p, s) for p, s in seeds[1:]]
    for s in sess[1:]:
        s.Preprocess()
    if timing:
        sess[0].ctx.timing_reset()
        sess[0].ctx.timing(2)
    ans, wall, on, mt = pm.search_loop_batched(sess, qs_per_session, k, 20, 3, ngroups, nthreads)
    kt = None
    if timing:
        sess[0].ctx.timing(False)
        kt = {n: sess[0].ctx.timing_get(n) for n in ("match_resolve", "answer", "prep_fold", "prep_offsets")}
    assert wall > 0 and (mt > 0).all()
    got = [(sess[i].counts(), sess[i].PIR.stats()) for i in range(len(seeds))]

    def run_oracle(i):   # one C call per phase: the oracle sessions run on host threads side by side
        p, s = seeds[i]
        o = oracle.Graph(v, graph, pir_seed=p, search_seed=s)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs_per_session[i], k, 20, 3)
        res = (oa, o.counts(), o.pir().stats())
        del o
        return res

    from concurrent.futures import ThreadPoolExecutor
    idx = list(range(len(seeds))) if check is None else list(check)
    with ThreadPoolExecutor(max_workers=min(oracle_workers, len(idx))) as ex:
        for i, (oa, oc, po) in zip(idx, ex.map(run_oracle, idx)):
            bad = np.where((ans[i] != oa).any(axis=1))[0]
            assert len(bad) == 0, (i, bad[:5].tolist())
            assert got[i][0] == oc, i
            ps = got[i][1]
            for key in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
                assert ps[key] == po[key], (i, key)
            assert ps["PrepCount"] >= 2, i
    return (ans, kt) if timing else ans


def test_search_sift1m_full_sessions(ctx, oracle):
    """configs[1] at full size: 1e6 SIFT-like vectors, d = 128, the reference's
    synthetic degree-32 graph (genRandomGraph), batch PIR over 1e6 x 640 B in
    16 partitions; four client sessions in two lock-step groups of the batched
    serving loop (the bench's driver), 26 queries each (window 23: every
    session re-preprocesses), k = 10, step 20, parallel 3.  Each session's
    answers, counters and maintenance equal an independent oracle run with
    its seeds."""
    from pacmann_amd.synth import random_graph, sift_like_vectors
    N = 1_000_000
    v = sift_like_vectors(N, 128, seed=100)
    graph = random_graph(N, 32, seed=200)
    rng = np.random.default_rng(3)
    seeds = [(11, 12), (21, 22), (31, 32), (41, 42)]
    qs = np.stack([np.clip(np.rint(v[rng.integers(0, N, 26)] + rng.normal(0, 8, (26, 128))), 0, 255)
                   .astype(np.float32) for _ in seeds])
    _sessions_vs_oracle(ctx, oracle, v, graph, qs, 10, seeds, ngroups=2, nthreads=4)


def test_search_msmarco_full_sessions(ctx, oracle):
    """MS-MARCO-shaped private search at full size (reproduce.sh:224-230:
    -n 3201821 -d 192 -m 32 -k 100 -step 20 -parallel 3): 3,201,821 vectors
    of d = 192 (per-dimension N(0, sigma_j)), a degree-32
    random graph, 896-B entries (CS 1,024 / SS 196); two sessions, 47 queries
    each (window 45: both re-preprocess), k = 100.  Answers, counters and
    maintenance equal independent oracle runs."""
    from pacmann_amd.synth import msmarco_like_vectors, random_graph
    N = 3_201_821
    v = msmarco_like_vectors(N, 192, seed=5)
    graph = random_graph(N, 32, seed=6)
    rng = np.random.default_rng(8)
    seeds = [(51, 52), (61, 62)]
    qs = np.stack([(v[rng.integers(0, N, 47)] + rng.normal(0, 0.1, (47, 192))).astype(np.float32)
                   for _ in seeds])
    _sessions_vs_oracle(ctx, oracle, v, graph, qs, 100, seeds, ngroups=1, nthreads=2)


def test_search_sift1m_full_shared_step(ctx, oracle):
    """The bench's serving kernels at full SIFT1M size: eight sessions in ONE
    lock-step group, so every round is one shared step over 8 x 16 = 128
    partitions -- the shapes that select k_match_resolve_s (match + resolve
    with the query sets expanded for k_answer_s) -- and the sessions'
    simultaneous re-preprocessing folds 8 clients per launch over mixed hint
    groups (k_prep_fold_rot).  Every session equals an independent oracle run."""
    from pacmann_amd.synth import random_graph, sift_like_vectors
    N = 1_000_000
    v = sift_like_vectors(N, 128, seed=101)
    graph = random_graph(N, 32, seed=201)
    rng = np.random.default_rng(13)
    seeds = [(110 + i, 210 + i) for i in range(8)]
    qs = np.stack([np.clip(np.rint(v[rng.integers(0, N, 26)] + rng.normal(0, 8, (26, 128))), 0, 255)
                   .astype(np.float32) for _ in seeds])
    _sessions_vs_oracle(ctx, oracle, v, graph, qs, 10, seeds, ngroups=1, nthreads=8)


def test_search_msmarco_full_shared_step(ctx, oracle):
    """MS-MARCO d=192 at full size through the shared step of eight sessions
    (128 partitions of CS 1,024 / SS 196 / E 112: k_match_resolve_s over 7,168
    hints, pre-expanded query sets, 8-client k_prep_fold_pipe), 47 queries each
    (every session re-preprocesses), k = 100.  Equal to independent oracle runs."""
    from pacmann_amd.synth import msmarco_like_vectors, random_graph
    N = 3_201_821
    v = msmarco_like_vectors(N, 192, seed=15)
    graph = random_graph(N, 32, seed=16)
    rng = np.random.default_rng(18)
    seeds = [(150 + i, 250 + i) for i in range(8)]
    qs = np.stack([(v[rng.integers(0, N, 47)] + rng.normal(0, 0.1, (47, 192))).astype(np.float32)
                   for _ in seeds])
    _sessions_vs_oracle(ctx, oracle, v, graph, qs, 100, seeds, ngroups=1, nthreads=8)


# ---------------------------------------------------------------------------
# the bench's serving shapes one group at a time (bench.py: SIFT1M 288
# sessions in 4 lock-step groups of 72 since the end of round 4, 64 before;
# MS-MARCO 64 sessions in 2 groups of 32; the whole SIFT1M shape:
# tests/test_gpu_headline.py)
# ---------------------------------------------------------------------------
def test_search_sift1m_bench_group_shape(ctx, oracle):
    """configs[1] at the bench's launch shapes: 64 sessions in ONE lock-step
    group over the full SIFT1M DB (1e6 x 640 B, 16 partitions each), so every
    round is one shared step over 64 x 16 = 1,024 partitions and 6,144
    sub-queries (k_match_resolve_s, k_answer_s with a grid of 6,144
    workgroups = 786,432 threads), and the 64 sessions' simultaneous
    maintenance after query 22 (window 23) folds all 64 clients in one
    k_prep_fold_rot launch (virtual hint groups mixing the clients).  24
    queries each, so every session re-preprocesses; all 64 sessions are
    replayed by independent oracle clients (pir.go:303-352, 354-471) and must
    equal them answer for answer, with equal counters."""
    from pacmann_amd.synth import random_graph, sift_like_vectors
    N, S = 1_000_000, 64
    v = sift_like_vectors(N, 128, seed=103)
    graph = random_graph(N, 32, seed=203)
    rng = np.random.default_rng(23)
    seeds = [(300 + i, 400 + i) for i in range(S)]
    qs = np.clip(np.rint(v[rng.integers(0, N, S * 24)] + rng.normal(0, 8, (S * 24, 128))), 0, 255)
    qs = qs.astype(np.float32).reshape(S, 24, 128)
    _, kt = _sessions_vs_oracle(ctx, oracle, v, graph, qs, 10, seeds, ngroups=1, nthreads=16, oracle_workers=16,
                                timing=True)
    # the launch shapes the bench measures actually ran
    n_ans, _, by = kt["answer"]
    assert n_ans == 24 * 20, n_ans             # one answer launch per shared step
    assert kt["match_resolve"][0] == n_ans     # the fused match + resolve each step
    assert by / n_ans > 300e6                  # 6,144 sub-queries x ~80.5 KB of answer bytes
    n_fold, _, fby = kt["prep_fold"]
    assert n_fold == 1 and fby > 60 * 15.8e9, (n_fold, fby)   # 64 clients' folds in one launch


def test_search_msmarco_bench_group_shape(ctx, oracle):
    """The MS-MARCO private-search block's launch shape: 32 sessions in ONE
    lock-step group (a shared step of 32 x 16 partitions of CS 1,024 / SS 196 /
    E 112, 3,072 sub-queries) over the full 3,201,821 x d = 192 DB, 47 queries
    each (window 45: every session re-preprocesses, the 32 clients folded in
    one launch), k = 100; every session equals an independent oracle run."""
    from pacmann_amd.synth import msmarco_like_vectors, random_graph
    N, S = 3_201_821, 32
    v = msmarco_like_vectors(N, 192, seed=25)
    graph = random_graph(N, 32, seed=26)
    rng = np.random.default_rng(28)
    seeds = [(500 + i, 600 + i) for i in range(S)]
    qs = (v[rng.integers(0, N, S * 47)] + rng.normal(0, 0.1, (S * 47, 192))).astype(np.float32).reshape(S, 47, 192)
    _, kt = _sessions_vs_oracle(ctx, oracle, v, graph, qs, 100, seeds, ngroups=1, nthreads=16, oracle_workers=8,
                                timing=True)
    n_ans, _, by = kt["answer"]
    assert n_ans == 47 * 20 and kt["match_resolve"][0] == n_ans
    assert kt["prep_fold"][0] == 1


# ---------------------------------------------------------------------------
# configs[2]: the MS-MARCO private-search block EXACTLY as bench.py serves it
# ---------------------------------------------------------------------------
def test_search_msmarco_bench_exact_shape(oracle):
    """bench.py private_search_msmarco, unchanged: the bench's data
    (msmarco_like_vectors(3,201,821, 192, seed=501)) and its GPU-built graph
    (pm.build_graph(v, 32, 1.2, seed=502): kNN + robustPrune), its queries
    (rng 503, 2 warm-up + 48 timed per session), 128 sessions (seeds 601 + i,
    602 + i), each on its own context, in 4 lock-step teams of 32 with 16
    pooled workers, k = 100, step 20, parallel 3, and the bench's two calls
    of the serving loop.  Every session reaches its maintenance after query
    44 (window 45, private-search.go:226-232) and the 128 clients are
    re-preprocessed as ONE launch set whose fold is ONE k_prep_fold_rot<1024>
    launch (CS 1,024: two chunks per staged block, 7 hints per lane) over all
    128 clients' virtual hint groups.  Nine sessions from all four teams are
    replayed by independent oracle clients over all 50 queries
    (pir.go:303-352, 354-471; search.go:114-234): answers, graph counts and
    FinishedBatchNum / QueriesMadeInPartition / PrepCount equal."""
    import pacmann_amd as pm
    from pacmann_amd.synth import msmarco_like_vectors
    N, DIM, K, S, G, NQ, WARM = 3_201_821, 192, 100, 128, 4, 50, 2
    ctx0 = pm.Context(0)
    v = msmarco_like_vectors(N, DIM, seed=501)
    g, _ = pm.build_graph(v, 32, 1.2, seed=502, ctx=ctx0)
    rng = np.random.default_rng(503)
    qs = (v[rng.integers(0, N, S * NQ)] + rng.normal(0, 0.1, (S * NQ, DIM))).astype(np.float32).reshape(S, NQ, DIM)
    base = pm.PIRGraphInfo(v, g, pir_seed=601, search_seed=602, ctx=ctx0)
    base.Preprocess()
    sess = [base] + [base.Session(601 + i, 602 + i, pm.Context(0)) for i in range(1, S)]
    for x in sess[1:]:
        x.Preprocess()
    ctxs = [x.ctx for x in sess]
    a0, _, _, _ = pm.search_loop_batched(sess, qs[:, :WARM], K, 20, 3, G, 16)
    for c in ctxs:
        c.sync()
        c.timing_reset()
        c.timing(2)
    a1, _, _, mt = pm.search_loop_batched(sess, qs[:, WARM:], K, 20, 3, G, 16)
    for c in ctxs:
        c.sync()
        c.timing(False)
    ans = np.concatenate([a0, a1], axis=1)

    def tsum(name):
        r = [c.timing_get(name) for c in ctxs]
        return tuple(sum(x[i] for x in r) for i in range(3))
    n_ans = tsum("answer")[0]
    assert n_ans == G * (NQ - WARM) * 20 and tsum("match_resolve")[0] == n_ans, n_ans
    assert tsum("host_dev_steps")[0] == n_ans   # the device loop chained every step (pm_drl.hip)
    assert tsum("host_prep_sets")[:2] == (1, S), tsum("host_prep_sets")
    n_fold, _, fby = tsum("prep_fold")
    sc = base.PIR.SubConfig(0)
    assert (sc["ChunkSize"], sc["SetSize"]) == (1024, 196)
    one = sum((base.PIR.SubConfig(p)["PrimaryHintNum"] + (base.PIR.SubConfig(p)["SetSize"] - 1) *
               base.PIR.SubConfig(p)["MaxQueryPerChunk"]) * base.PIR.SubConfig(p)["SetSize"] * 112 * 8
              for p in range(16))
    assert n_fold == 1 and abs(fby / one - S) < 0.5, (n_fold, fby / one)
    assert tsum("host_fold_rot1024")[0] == 1 and tsum("host_fold_other")[0] == 0
    assert (mt > 0).all()
    check = [0, 1, 31, 32, 50, 64, 95, 96, 127]   # teams of 32: 0-31, 32-63, 64-95, 96-127
    got = {i: (sess[i].counts(), sess[i].PIR.stats()) for i in check}
    del sess, base, ctxs

    def run_oracle(i):
        o = oracle.Graph(v, g, pir_seed=601 + i, search_seed=602 + i)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], K, 20, 3)
        res = (oa, o.counts(), o.pir().stats())
        del o
        return res
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=8) as ex:
        for i, (oa, oc, po) in zip(check, ex.map(run_oracle, check)):
            bad = np.where((ans[i] != oa).any(axis=1))[0]
            assert len(bad) == 0, (i, bad[:5].tolist())
            assert got[i][0] == oc, i
            for key in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
                assert got[i][1][key] == po[key], (i, key)
            assert got[i][1]["PrepCount"] == 2, i


def test_group_preprocessing_msmarco_64_clients(ctx, oracle):
    """pm_batchpir_group_preprocessing at the MS-MARCO bench's maintenance
    shape: 64 clients of the 3,201,821 x 896 B server (CS 1,024 / SS 196)
    folded in ONE k_prep_fold_rot<1024> launch (virtual hint groups mixing the
    clients) give, for every client and sampled partitions, exactly the state
    of that client's own Preprocessing, through two epochs; clients 0 and 63
    also equal independent oracle clients after the first grouped epoch."""
    import pacmann_amd as pm
    N, E, B, K = 3_201_821, 112, 32, 64
    db = rand_db(N, E, seed=65)
    server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    server.Preprocessing()
    cg, ci = pm.Context(0), pm.Context(0)
    seeds = [3000 + i for i in range(K)]
    grouped = [server.Client(sd, cg) for sd in seeds]
    alone = [server.Client(sd, ci) for sd in seeds]
    for c in grouped + alone:
        c.Preprocessing()   # epoch 0, one client at a time
    grp = pm.BatchPIRGroup(grouped)
    for epoch in (1, 2):
        cg.timing_reset()
        cg.timing(1)
        grp.Preprocessing()
        cg.sync()
        cg.timing(False)
        assert cg.timing_get("host_fold_rot1024")[0] == 1 and cg.timing_get("prep_fold")[0] == 1, epoch
        for c in alone:
            c.Preprocessing()
        for i in range(K):   # one partition per client (all 16 covered), four for every 8th
            for p in ((i % 16,) if i % 8 else (0, 5, 10, 15)):
                diff = state_diff(grouped[i].export_state(p), alone[i].export_state(p))
                assert not diff, (epoch, i, p, diff)
        assert grouped[0].stats()["PrepCount"] == alone[0].stats()["PrepCount"] == epoch + 1
        if epoch == 1:
            for i in (0, K - 1):
                o = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=seeds[i])
                o.Preprocessing()   # epoch 0
                o.Preprocessing()   # epoch 1
                for p in (0, 7, 15):
                    diff = state_diff(grouped[i].export_state(p), o.sub(p).export_state())
                    assert not diff, (i, p, diff)
                del o


# ---------------------------------------------------------------------------
# configs[1]: the serving loop's maintenance fold of 64 clients in one launch
# ---------------------------------------------------------------------------
def test_group_preprocessing_sift1m_64_clients(ctx):
    """pm_batchpir_group_preprocessing at the bench's group shape: 64 SIFT1M
    clients (1e6 x 640 B, CS 512 / SS 124) folded in ONE k_prep_fold_rot launch
    (virtual hint groups mixing clients) give, for every client and sampled
    partitions, exactly the state of that client's own Preprocessing (the
    single-client fold, oracle-checked in test_gpu_parity), through two
    epochs."""
    import pacmann_amd as pm
    N, E, B, K = 1_000_000, 80, 32, 64
    db = rand_db(N, E, seed=64)
    server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    server.Preprocessing()
    cg, ci = pm.Context(0), pm.Context(0)
    seeds = [1000 + i for i in range(K)]
    grouped = [server.Client(sd, cg) for sd in seeds]
    alone = [server.Client(sd, ci) for sd in seeds]
    for c in grouped + alone:
        c.Preprocessing()   # epoch 0, one client at a time
    grp = pm.BatchPIRGroup(grouped)
    ctx.timing_reset()
    for epoch in (1, 2):
        grp.Preprocessing()
        for c in alone:
            c.Preprocessing()
        for i in range(K):
            for p in ((0, 15) if i % 8 else (0, 5, 10, 15)):
                diff = state_diff(grouped[i].export_state(p), alone[i].export_state(p))
                assert not diff, (epoch, i, p, diff)
        assert grouped[0].stats()["PrepCount"] == alone[0].stats()["PrepCount"] == epoch + 1


# ---------------------------------------------------------------------------
# configs[3] / configs[4]: the sharded private graph search at full size, every
# record checked (pm_set_option "verify_records": the loop checks each
# answered record against the graph's spec and the reference-order L2 on the
# host, and explains each unanswered id)
# ---------------------------------------------------------------------------
def _bigann_search_checked(ctx, n, shard, nshards, model_peers, S=4, Q=12):
    import pacmann_amd as pm
    base = pm.PIRGraphInfo.Synthetic(n, 128, 32, data_seed=51, shard=shard, nshards=nshards, pir_seed=61,
                                     search_seed=62, ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(61 + i, 62 + i, pm.Context(0)) for i in range(1, S)]
    for x in sess[1:]:
        x.Preprocess()
    qs = np.random.default_rng(63).random((S, Q, 128), dtype=np.float32)   # genRandomMatrix queries
    for x in sess:
        x.ctx.timing_reset()
    pm.set_option("verify_records", 1)
    try:
        ans, _, _, _ = pm.search_loop_sharded(sess, qs, 10, 20, 3, 2, 8, model_peers=model_peers)
    finally:
        pm.set_option("verify_records", 0)

    def cnt(name):
        return sum(x.ctx.timing_get("host_records_" + name)[0] for x in sess)
    c = {k: cnt(k) for k in ("verified", "bad", "dropped", "failed", "peer", "unexplained")}
    fetched = sum(x.counts()[0] for x in sess)
    assert fetched == S * Q * 20 * 96
    assert sum(c.values()) == fetched, c               # every record of every round was checked
    assert c["bad"] == 0 and c["unexplained"] == 0 and c["peer"] == 0, c
    assert c["verified"] > 0.6 * fetched, c            # most ids are answered (the rest: overflow, 2^-8 no-hits)
    assert c["failed"] <= 0.02 * fetched, c
    assert sum(x.counts()[1] for x in sess) == c["verified"]   # the reference's success count agrees
    assert (ans >= 0).all()
    return c


def test_sharded_search_bigann_100m_full_size_records(ctx):
    """configs[3] as the bench serves it on one GPU: the 100M-vertex synthetic
    graph DB (64 GB generated on the device, CS 8,192 / SS 764 partitions),
    one rank holding all partitions, 4 sessions in 2 lock-step teams, 12
    queries each (k 10, step 20, parallel 3): all 92,160 records checked."""
    _bigann_search_checked(ctx, 100_000_000, 0, 1, False)


def test_sharded_search_bigann_1b_shard0_full_size_records(ctx):
    """configs[4]: shard 0 of the 1B-vertex graph's 8-way layout (partitions 0
    and 8, 80 GB generated on the device, CS 16,384 / SS 3,816) with the other
    shards' records generated from the spec (modelled peers): every record the
    loop consumed — this shard's PIR answers and the modelled ones — equals
    the graph's row and the reference-order L2, and every unanswered id is an
    overflow drop or a failed sub-query of this shard."""
    _bigann_search_checked(ctx, 1_000_000_000, 0, 8, True)
