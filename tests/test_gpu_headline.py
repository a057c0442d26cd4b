"""GPU parity at the exact configuration of the headline bench line
(bench.py main(), BASELINE.json configs[1]), query stream included:

  * the bench's data: `sift_like_vectors(1e6, 128, seed=100)` and the graph
    `pm.build_graph(v, 32, 1.2, seed=7)` built on the GPU (kNN + robustPrune);
  * the bench's serving shape: 288 sessions in 4 lock-step teams of 72
    (pm_search_loop_batched -> run_batched_dev: each team's rounds chained on
    its stream by the device loop, pm_drl.hip), every round of a team ONE
    shared step over 72 x 16 partitions;
  * the merged maintenance: the 288 sessions reach their re-preprocessing at
    the same query (window 23, private-search.go:226-232), and the waiting
    teams' clients are re-preprocessed as ONE launch set (one k_prep_fold_rot
    launch for all 288 clients);
  * the bench's queries: `make_queries(v, S * 57 + 64, seed=300)` cut into
    57 per session, of which the bench serves 5 warm-up queries and then its
    20-query timed region in two calls -- the same two calls here (25 queries
    per session, past the trigger), k 10, step 20, parallel 3.

Sixteen sessions spread over all four teams are replayed by independent
oracle clients with the same seeds and queries (pir.go:303-352 preprocessing,
pir.go:354-471 queries, search.go:114-234 beam search): answers, graph counts
and the batch-PIR counters must be equal."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, DIM, M, K, STEP, PAR = 1_000_000, 128, 32, 10, 20, 3
S, TEAMS, THREADS = 288, 4, 16   # bench.py SESSIONS, lockstep teams, threads
WARMUP, STEPS, NQ = 5, 20, 5 + 20 + 24 + 8   # bench.py defaults: --warmup, --steps, + KT_QUERIES + PROFILE_QUERIES
QUERIES = WARMUP + STEPS
CHECK = [0, 1, 37, 71, 72, 73, 100, 143, 144, 150, 200, 215, 216, 250, 286, 287]


def test_headline_bench_sessions_4_teams_vs_oracle(oracle):
    import pacmann_amd as pm
    from pacmann_amd.synth import sift_like_vectors
    ctx0 = pm.Context(0)
    v = sift_like_vectors(N, DIM, seed=100)              # bench.py make_data, rank 0
    g, _ = pm.build_graph(v, M, 1.2, seed=7, ctx=ctx0)  # the GPU-built graph the bench serves
    import importlib.util
    import pathlib
    spec = importlib.util.spec_from_file_location("pm_bench", pathlib.Path(__file__).resolve().parents[1] / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert (bench.SESSIONS, bench.KT_QUERIES, bench.PROFILE_QUERIES) == (S, 24, 8)
    qsess = bench.make_queries(v, S * NQ + 64, seed=300)[:S * NQ].reshape(S, NQ, DIM)   # bench.py main, rank 0
    qs = np.ascontiguousarray(qsess[:, :QUERIES])
    seeds = [(11 + i, 12 + i) for i in range(S)]         # bench.py: 11 + 97 * rank + i, 12 + 97 * rank + i
    base = pm.PIRGraphInfo(v, g, pir_seed=seeds[0][0], search_seed=seeds[0][1], ctx=ctx0)
    base.Preprocess()
    sess = [base] + [base.Session(p, s_, pm.Context(0)) for p, s_ in seeds[1:]]
    for x in sess[1:]:
        x.Preprocess()
    ctxs = [x.ctx for x in sess]
    for c in ctxs:
        c.timing_reset()
        c.timing(2)
    a0, _, _, mt0 = pm.search_loop_batched(sess, np.ascontiguousarray(qs[:, :WARMUP]), K, STEP, PAR, TEAMS, THREADS)
    a1, wall, _, mt = pm.search_loop_batched(sess, np.ascontiguousarray(qs[:, WARMUP:]), K, STEP, PAR, TEAMS, THREADS)
    ans = np.concatenate([a0, a1], axis=1)   # the bench's warm-up call, then its timed region
    for c in ctxs:
        c.sync()
        c.timing(False)

    def tsum(name):
        r = [c.timing_get(name) for c in ctxs]
        return tuple(sum(x[i] for x in r) for i in range(3))
    # the launch shapes of the bench line: every shared step of every team is one
    # k_match_resolve_s + one k_answer_p over 72 sessions' partitions ...
    n_ans, _, by = tsum("answer")
    assert n_ans == TEAMS * QUERIES * STEP, n_ans
    assert tsum("match_resolve")[0] == n_ans
    assert by / n_ans > 330e6   # ~6,912 sub-queries x ~80.5 KB per step (minus cache hits)
    # ... every one of them chained on the GPU by the device loop (pm_drl.hip)
    assert tsum("host_dev_steps")[0] == n_ans and tsum("host_dev_queries")[1] == S * QUERIES
    # ... and the maintenance ran ONCE, merged: one launch set of all 288
    # clients, one fold launch over all their hints
    sets, clients, _ = tsum("host_prep_sets")
    assert (sets, clients) == (1, S), (sets, clients)
    n_fold, _, fby = tsum("prep_fold")
    one = 0
    for p in range(16):
        c = base.PIR.SubConfig(p)
        one += (c["PrimaryHintNum"] + (c["SetSize"] - 1) * c["MaxQueryPerChunk"]) * c["SetSize"] * 80 * 8
    assert n_fold == 1 and abs(fby / one - S) < 0.5, (n_fold, fby / one)
    assert (mt > 0).all() and wall > 0
    got = {i: (sess[i].counts(), sess[i].PIR.stats()) for i in CHECK}
    del sess, base, ctxs   # free the 288 clients' device state before the oracle runs

    def run_oracle(i):
        p, s_ = seeds[i]
        o = oracle.Graph(v, g, pir_seed=p, search_seed=s_)
        o.Preprocess()
        oa, _, _ = o.SearchLoop(qs[i], K, STEP, PAR)
        res = (oa, o.counts(), o.pir().stats())
        del o
        return res
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=16) as ex:
        for i, (oa, oc, po) in zip(CHECK, ex.map(run_oracle, CHECK)):
            bad = np.where((ans[i] != oa).any(axis=1))[0]
            assert len(bad) == 0, (i, bad[:5].tolist())
            assert got[i][0] == oc, i
            for key in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
                assert got[i][1][key] == po[key], (i, key)
            assert got[i][1]["PrepCount"] == 2, i
