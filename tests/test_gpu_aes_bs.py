"""The bitsliced PRF tables (k_prep_offsets_bs, pm_aes_bs.h; round 6) against
the oracle.

pm_set_option("aes_bs", 1) makes every preprocessing build its PRF tables
(tabT, the hint-search table, and the chunk-major table where the fold
stages it) with the bitsliced VALU AES instead of the T-table form.  The
client state after preprocessing, and every answer and state of a query
sequence that reads those tables (hint search, set expansion, refresh), must
equal the oracle bit for bit (Client.Preprocessing / Client.Query,
pianopir/pir.go:267-471; AES-128-MMO, pianopir/aes_amd64.s:51-82).  The
shapes cover ChunkSize 16 to 2,048 (a hint count that is not a multiple of 32,
so a bitsliced lane's tail tags, at CS 16), SetSize % 8 == 4 (padding tiles),
and the multi-client group preprocessing of the batched serving.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 20240501
STATE_KEYS = ["round_keys", "primary_tag", "primary_parity", "primary_pp", "backup_tag",
              "backup_parity", "repl_idx", "repl_val", "hist"]


@pytest.fixture
def aes_bs():
    import pacmann_amd as pm
    pm.set_option("aes_bs", 1)
    try:
        yield
    finally:
        pm.set_option("aes_bs", -1)


def rand_db(n, e, seed=1):
    return np.random.default_rng(seed).integers(0, 2**64, size=n * e, dtype=np.uint64)


@pytest.mark.parametrize("N,E,F", [(60, 4, 8), (5000, 6, 8), (18750, 4, 40), (62500, 80, 8), (100_000, 8, 8),
                                   (1_000_000, 4, 8)])
def test_prep_offsets_bs_state(ctx, oracle, aes_bs, N, E, F):
    import pacmann_amd as pm
    db = rand_db(N, E, seed=N + 7)
    g = pm.PianoPIR(N, E * 8, db, F, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, F, seed=SEED)
    assert g.Config() == o.Config()
    g.Preprocessing()
    o.Preprocessing()
    a, b = g.export_state(), o.export_state()
    for k in STATE_KEYS:
        assert np.array_equal(a[k], b[k]), k


@pytest.mark.parametrize("N,E,F", [(60, 4, 8), (18750, 4, 40), (62500, 8, 8)])
def test_prep_offsets_bs_query_sequence(ctx, oracle, aes_bs, N, E, F):
    """Every query of a client's budget (through its own re-preprocessing at
    FinishedQueryNum == MaxQueryNum, pir.go:527-530) reads the bitsliced
    tables: responses, statuses and the final state equal the oracle's."""
    import pacmann_amd as pm
    db = rand_db(N, E, seed=N + 9)
    g = pm.PianoPIR(N, E * 8, db, F, seed=SEED, ctx=ctx)
    o = oracle.PianoPIR(N, E * 8, db, F, seed=SEED)
    g.Preprocessing()
    o.Preprocessing()
    rng = np.random.default_rng(N)
    ids = rng.integers(0, N, size=int(g.Config()["MaxQueryNum"]) + 20)
    ids[5::17] = ids[3]   # repeats exercise the local cache
    for i, idx in enumerate(ids):
        real = (i % 11) != 4
        got, err = g.Query(int(idx), real)
        want, st = o.Query(int(idx), real)
        assert (err.code if err else 0) == st, i
        assert np.array_equal(got, want), i
    assert g.Config()["FinishedQueryNum"] == o.Config()["FinishedQueryNum"]
    a, b = g.export_state(), o.export_state()
    for k in STATE_KEYS:
        assert np.array_equal(a[k], b[k]), k


def test_prep_offsets_bs_group(ctx, oracle, aes_bs):
    """Five clients of one server through the group query (one merged
    multi-client preprocessing per trigger): entries, flags and counters equal
    independent oracle clients through the batch layer's re-preprocessing."""
    import pacmann_amd as pm
    N, E, B = 30_000, 8, 8
    db = rand_db(N, E, 95)
    server = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=SEED, ctx=ctx)
    server.Preprocessing()
    seeds = [SEED, 31, 32, 33, 34]
    clients = [server] + [server.Client(sd, pm.Context(0)) for sd in seeds[1:]]
    for c in clients[1:]:
        c.Preprocessing()
    grp = pm.BatchPIRGroup(clients)
    ors = [oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=sd) for sd in seeds]
    for o in ors:
        o.Preprocessing()
    rng = np.random.default_rng(25)
    maxq = server.SubConfig(0)["MaxQueryNum"]
    for b in range(int(maxq // 3) + 6):
        q = rng.integers(0, N, size=(len(clients), 3 * B), dtype=np.uint64)
        out, ok = grp.QueryWithMask(q)
        for i, o in enumerate(ors):
            want, _ = o.Query(q[i])
            assert np.array_equal(out[i], want), (b, i)
    for c, o in zip(clients, ors):
        for k in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
            assert c.stats()[k] == o.stats()[k], k
        assert c.stats()["PrepCount"] > 1
