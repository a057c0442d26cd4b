"""bench.py — private queries/sec on the SIFT1M-shaped private search (1 MI355X per rank).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--sessions S] [--no-cpu-baseline] [--no-config2]

Workload (BASELINE.json configs[1], the metric's config): n = 1e6 vectors,
d = 128, degree m = 32 graph, k = 10, step = 20, parallel = 3, batch PIR with
BatchSize = m = 32 (16 partitions) and FailureProbLog2 = 8, exactly the
private-search.go harness (run-private-search.sh flags).  Data are synthetic
(no dataset in the image): a clustered SIFT-like mixture with integer values in
[0,255] and a degree-32 graph built on the GPU (exact kNN + robustPrune; --graph
random: the reference's genRandomGraph, private-search.go:54-69).

Serving: one GPU serves S client sessions at once (--sessions, default 288).
Every session is a full PianoPIR client (own keys, hint state, cache,
maintenance) over the one server DB on the device.  Default (--mode batched,
pm_search_loop_batched): the sessions run in G lock-step groups (--groups,
default 4 = the process's hardware queues); every batch-PIR round of a group's
sessions is ONE shared step over their S/G x 16 partitions, and 16 host worker
threads (--threads) run the sessions' searches between steps, so one group's
step overlaps the others' host work.  --mode concurrent: each session on its
own host thread and stream with its own step launches (pm_search_loop_sessions).  One step = one private query per
session (GraphANNFrontend.SearchKNN over PIRGraphInfo, 20 batch-PIR rounds of
96 ids) plus, whenever the harness trigger fires (private-search.go:226-232),
that session's full hint re-preprocessing — so `value` is all sessions'
queries / wall time including maintenance, the reference's own accounting
summed over clients.  `single_session` reports one client alone (latency view).

Multi-GPU: one process per GPU (torch.distributed.run); every rank runs its
own server replica and S sessions on its own GPU and query streams (queries
are independent units, no data-path exchange), so scaling is weak and `value`
is the sum of queries over the max of the ranks' times.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

N, DIM, M, K_TOP, STEP, PARALLEL, F = 1_000_000, 128, 32, 10, 20, 3, 8
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# LDS ceilings (MI355X_MICROARCH.md §LDS: 64 x 4-B banks; every CU streaming at
# ~2.4 GHz): ds_read_b64 / b128 ~150 TB/s (256 B/clk/CU), ds_read_b32 ~75 TB/s
# (128 B/clk/CU, 32 lookups/clk/CU when conflict-free)
LDS_B128_PEAK_GBS, LDS_B32_PEAK_GBS = 150_000.0, 75_000.0
# k_prep_offsets' AES (pm_aes.h prf_lo16_split): rounds 2-8 16 T-table lookups
# each, round 9 two columns (8), round 10 two S-box bytes (2), round 1's
# per-hint half (4 per 8 chunks) = 122.5 conflict-free ds_read_b32 per PRF
# (the tables are 32x bank-replicated), and ~2 VALU per lookup (v_perm address,
# v_bitop3 XORs, one rotation per column)
AES_LOOKUPS_PER_PRF = 122.5
# SetSize <= 256 (SIFT1M, MS-MARCO): round 2 hoisted per hint (pm_aes.h r2_hint):
# round 2 takes 4 lookups per PRF + 12 per hint per 8 chunks = 112 per PRF
AES_LOOKUPS_PER_PRF_R2 = 112.0


def prf_peak_g(lookups: float) -> float:
    """The T-table lookup ceiling in G PRF/s (conflict-free ds_read_b32)."""
    return LDS_B32_PEAK_GBS * 1e9 / 4 / lookups / 1e9


PRF_PEAK_G = prf_peak_g(AES_LOOKUPS_PER_PRF)   # ~153 G PRF/s
METRIC = "private queries/sec + PIR-scan HBM GB/s, SIFT1M d=128 at 1/2/4/8 GPUs"
PREP_KERNELS = ["prep_offsets", "prep_fold", "prep_repl", "l2_rows"]
STEP_KERNELS = ["step", "hint_match", "resolve", "match_resolve", "gather", "answer",
                "team_round"]   # timed in the measured region too (team_round: the device loop's round, pm_drl.hip)
KERNELS = PREP_KERNELS + STEP_KERNELS
PROFILE_QUERIES = 8
# the kernel-timing pass after the timed region (same sessions, teams and
# launch shapes; events on every launch): 24 queries, so it holds one
# maintenance of every session (window 23 queries, private-search.go:226-232)
KT_QUERIES = 24
SESSIONS = 288  # client sessions per GPU, 4 teams of 72 (round 4 ABBA, one box: 256: 16.8K q/s, 288: 17.3K, 320: 17.3K)
GROUPS = 4      # lock-step groups (GPU_MAX_HW_QUEUES = 4 hardware queues per process)
THREADS = 16    # host worker threads of the batched loop (the box gives a GPU 16 host cores)
SYMBOLS = {"prep_fold": "void pm::k_prep_fold_rot<512>(pm::PmPart const*, unsigned int, unsigned int, unsigned int, "
                        "unsigned int, unsigned int, unsigned int, unsigned int)",
           "answer": None, "step": "void pm::k_step<2>(pm::PmStep)", "resolve": "void pm::k_resolve<true>(pm::PmStep)",
           "hint_match": "pm::k_match(pm::PmStep)", "prep_offsets": "pm::k_prep_offsets(pm::PmPart const*)",
           "gather": "void pm::k_gather<2>(pm::PmStep)",
           "match_resolve": "void pm::k_match_resolve_s<2, 256>(pm::PmStep)"}
# the server answer of search-sized shapes: the small-LDS instance with
# PM_ANSWER_NT threads per workgroup (pm_query.hip step_answer; 0: generic)
ANSWER_NT = int(os.environ.get("PM_ANSWER_NT", "128"))
ANSWER_BLOCK = ANSWER_NT or 512
SYMBOLS["answer"] = (f"void pm::k_answer_s<2, {ANSWER_NT}>(pm::PmStep)" if ANSWER_NT
                     else "void pm::k_answer<2>(pm::PmStep)")
# the batched steps' answer (>= 512 sub-queries with pre-expanded query sets):
# k_answer_p, two sub-queries per 128-thread workgroup (PM_ANSWER_PAIR=0: k_answer_s)
ANSWER_PAIR = os.environ.get("PM_ANSWER_PAIR", "1") != "0"
if ANSWER_PAIR:
    SYMBOLS["answer"] = "void pm::k_answer_p<2, 128>(pm::PmStep)"


def answer_grid(nsub: int) -> int:
    """Work-items of the answer launch of a shared step of nsub sub-queries."""
    return (nsub + 1) // 2 * 128 if ANSWER_PAIR and nsub >= 512 else nsub * ANSWER_BLOCK
HOST = ["host_search_knn", "host_knn_init", "host_knn_final", "host_knn_batch", "host_knn_update",
        "host_gvi_parse", "host_batch_query", "host_step_launch", "host_step_wait", "host_step_post",
        "host_wait_first_token", "host_wait_all_tokens", "host_rows_seen", "host_rows_torn", "host_wait_done"]


T_START = time.perf_counter()


def progress(msg: str):
    """One line per phase on stderr (long profiler runs show they are alive)."""
    print(f"[bench {time.perf_counter() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def make_data(rank: int, graph: str, ctx):
    """SIFT1M-shaped synthetic vectors and the degree-32 graph: built on the GPU
    (pm_build_graph: BuildGraph with exact kNN candidates in place of NGT), or
    the reference's synthetic-mode genRandomGraph (--graph random)."""
    import pacmann_amd as pm
    from pacmann_amd.synth import random_graph, sift_like_vectors
    v = sift_like_vectors(N, DIM, seed=100 + rank)
    if graph == "random":
        return v, random_graph(N, M, seed=200 + rank), None
    ctx.sync()
    t0 = time.perf_counter()
    g, tm = pm.build_graph(v, M, 1.2, seed=7 + rank, ctx=ctx)
    tm = {k: round(x, 4) for k, x in tm.items()}
    tm["total_s"] = round(time.perf_counter() - t0, 4)
    return v, g, tm


def make_queries(v, n, seed):
    rng = np.random.default_rng(seed)
    idx = rng.integers(0, v.shape[0], size=n)
    q = v[idx] + rng.normal(0, 8, size=(n, v.shape[1])).astype(np.float32)
    return np.clip(np.rint(q), 0, 255).astype(np.float32)


def pmc_traffic(kernel_symbol: str, grid: int | None = None):
    """Memory-side bytes per dispatch of `kernel_symbol` (of launches of `grid`
    threads if given) from the newest committed rocprofv3 PMC summary
    (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, collected in separate --pmc
    passes of this bench); None if absent.  These count the L2's requests to
    the fabric, Infinity Cache hits included (MI355X_MICROARCH.md): an upper
    bound on HBM bytes."""
    best = None
    for f in sorted((ROOT / "profiles").glob("r*/pmc_summary.json")):
        k = json.loads(f.read_text()).get("kernels", {}).get(kernel_symbol)
        if k and grid is not None:
            k = k.get("by_grid", {}).get(str(grid))
        if k and "hbm_bytes_per_dispatch_corrected" in k:
            best = (k["hbm_bytes_per_dispatch_corrected"], str(f.relative_to(ROOT)))
    return best


def attach_traffic(roof: dict | None, symbol: str, grid: int) -> None:
    """roof["traffic"]: PMC HBM bytes per dispatch of `symbol` at launch shape
    `grid` (threads) from the committed profiles (pmc_traffic), with its source."""
    if not roof:
        return
    tr = pmc_traffic(symbol, grid)
    roof["traffic"], roof["traffic_source"] = (tr[0], tr[1]) if tr else (None, None)
    roof["symbol"], roof["grid_threads"] = symbol, grid


# BASELINE.json configs[2]: MS-MARCO-shaped batch PIR, the TestBatchPIRPerf
# shape (pianopir/pir_test.go:204-275): 3,201,821 entries of 112 words, BatchSize
# 32, FailureProbLog2 8, 300 batches of 32 uniform ids.
C2_N, C2_E, C2_B, C2_BATCHES = 3_201_821, 112, 32, 300
C2_CLIENTS = 32   # clients of the server answered together (one shared step per round)


def step_grid_threads(nsub, npart):
    """k_step's launch (pmk::step_fused) for nsub sub-queries over npart
    partitions, in threads: match, resolve and answer workgroups plus the
    gather helpers pm_engine.cpp engine_step adds while the launch fits 240
    co-resident 1,024-thread workgroups (PM_STEP_HELP, default 3, at most 3)."""
    cap = int(os.environ.get("PM_STEP_HELP", "3"))
    base = 2 * nsub + npart
    nhelp = min(3, max(cap, 0), (240 - base) // nsub) if base < 240 else 0
    return (base + nhelp * nsub) * 1024


def batch_pir_msmarco(ctx, with_cpu: bool):
    """Preprocessing time, then batch-query throughput, of the batch-PIR path at
    the configs[2] shape, with the step kernel's answer-bytes roofline."""
    import pacmann_amd as pm
    db = np.random.default_rng(77).integers(0, 2**64, size=C2_N * C2_E, dtype=np.uint64)
    g = pm.SimpleBatchPianoPIR(C2_N, C2_E * 8, C2_B, db, 8, seed=21, ctx=ctx)
    ctx.sync()
    t0 = time.perf_counter()
    g.Preprocessing()
    ctx.sync()
    prep = time.perf_counter() - t0
    rng = np.random.default_rng(78)
    batches = rng.integers(0, C2_N, size=(2 * C2_BATCHES + 10, C2_B)).astype(np.uint64)
    rows = db.reshape(C2_N, C2_E)
    for b in batches[:10]:   # warm-up
        g.Query(b)
    ctx.sync()

    def query_pass(bs):
        """The reference's loop (pir_test.go:245-262): Query, then check the
        first response (zero or the entry).  Returns (seconds, mismatches)."""
        t0 = time.perf_counter()
        bad = 0
        for b in bs:
            resp, _ = g.Query(b)
            r0 = resp[0]
            bad += int(r0.any() and not np.array_equal(r0, rows[int(b[0])]))
        ctx.sync()
        return time.perf_counter() - t0, bad

    # the throughput pass runs uninstrumented: events in the step's dispatch
    # packet add ~8 us of launch time per batch (tools/batchpir_host.py), so
    # the step kernel is timed over a second pass of fresh batches
    support0 = g.SupportBatchNum
    online, bad = query_pass(batches[10:10 + C2_BATCHES])
    ctx.timing_reset()
    ctx.timing(2)
    online_timed, bad_t = query_pass(batches[10 + C2_BATCHES:])
    ctx.timing(False)
    n, ms, by = ctx.timing_get("step")
    out = {"workload": "TestBatchPIRPerf shape (configs[2], MS-MARCO 3.2M): 3,201,821 x 896 B, BatchSize 32, "
                       "FailureProbLog2 8, uniform synthetic DB and ids",
           "preprocessing_s": round(prep, 6), "batches": C2_BATCHES,
           "batch_queries_per_s": round(C2_BATCHES / online, 1),
           "ids_per_s": round(C2_BATCHES * C2_B / online, 1), "ms_per_batch": round(online / C2_BATCHES * 1e3, 4),
           "first_response_mismatches": bad + bad_t,
           "kernel_timing_pass": {"batches": C2_BATCHES, "ms_per_batch": round(online_timed / C2_BATCHES * 1e3, 4),
                                  "note": "a second pass of fresh batches with the step kernel's events on"},
           "support_batch_num": support0, "finished_batch_num": g.FinishedBatchNum}
    if n:
        ach = (by / n) / (ms / n / 1e3) / 1e9
        out["roofline"] = {"bound": "hbm", "kernel": "step", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "avg_ms": round(ms / n, 5),
                           "launches": n, "alg_bytes_per_launch": by / n,
                           "note": "k_step of one 32-id batch (32 sub-queries over 16 partitions: latency-bound, "
                                   "one workgroup per sub-query gathers 196 rows); every launch of the timed batches"}
        attach_traffic(out["roofline"], SYMBOLS["step"], step_grid_threads(C2_B, 16))
    # C2_CLIENTS clients of the one server DB, every batch of all of them answered
    # together (pm_batchpir_group_*: one shared step per round)
    clients = [g] + [g.Client(1000 + i, pm.Context(0)) for i in range(C2_CLIENTS - 1)]
    for c in clients[1:]:
        c.Preprocessing()
    grp = pm.BatchPIRGroup(clients)
    gb = rng.integers(0, C2_N, size=(2 * C2_BATCHES + 10, C2_CLIENTS, C2_B)).astype(np.uint64)
    for b in gb[:10]:
        grp.QueryWithMask(b)
    for c in clients:
        c.ctx.sync()

    def group_pass(bs):
        t0 = time.perf_counter()
        bad = 0
        for b in bs:
            resp, ok = grp.QueryWithMask(b)
            r0, ids0 = resp[:, 0], b[:, 0].astype(np.int64)   # every client's first response: zero or its entry
            bad += int(((r0 != rows[ids0]).any(axis=1) & ok[:, 0]).sum() + (r0[~ok[:, 0]] != 0).any())
        for c in clients:
            c.ctx.sync()
        return time.perf_counter() - t0, bad

    # throughput uninstrumented, then the kernels timed over fresh rounds (as above)
    gon, gbad = group_pass(gb[10:10 + C2_BATCHES])
    clients[0].ctx.timing_reset()
    clients[0].ctx.timing(2)   # the shared steps run on the first client's stream
    gon_t, gbad_t = group_pass(gb[10 + C2_BATCHES:])
    clients[0].ctx.timing(False)
    out["clients_grouped"] = {"clients": C2_CLIENTS, "batches_per_client": C2_BATCHES,
                              "batch_queries_per_s": round(C2_CLIENTS * C2_BATCHES / gon, 1),
                              "ids_per_s": round(C2_CLIENTS * C2_BATCHES * C2_B / gon, 1),
                              "ms_per_round": round(gon / C2_BATCHES * 1e3, 4),
                              "first_response_mismatches": gbad + gbad_t,
                              "kernel_timing_pass_ms_per_round": round(gon_t / C2_BATCHES * 1e3, 4)}
    n, ms, by = clients[0].ctx.timing_get("answer")
    if n:
        ach = (by / n) / (ms / n / 1e3) / 1e9
        out["clients_grouped"]["roofline"] = {
            "bound": "hbm", "kernel": "answer", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 4), "avg_ms": round(ms / n, 5), "launches": n,
            "alg_bytes_per_launch": by / n,
            "kernel_avg_us": {k: round(v[1] / v[0] * 1e3, 3) for k, v in
                              ((k, clients[0].ctx.timing_get(k)) for k in ("hint_match", "resolve", "match_resolve", "answer")) if v[0]}}
        # (the grouped batch PIR's steps take k_match_part8 -> k_resolve -> k_answer_s: no pre-expanded sets)
        attach_traffic(out["clients_grouped"]["roofline"], f"void pm::k_answer_s<2, {ANSWER_NT}>(pm::PmStep)",
                       C2_CLIENTS * C2_B * ANSWER_BLOCK)
    del grp, clients
    if with_cpu:
        from oracle import oracle as O
        o = O.SimpleBatchPianoPIR(C2_N, C2_E * 8, C2_B, db, 8, seed=21)
        t0 = time.perf_counter()
        o.Preprocessing()
        oprep = time.perf_counter() - t0
        t0 = time.perf_counter()
        for b in batches[10:10 + C2_BATCHES]:
            o.Query(b)
        oon = time.perf_counter() - t0
        out["cpu_baseline"] = {"preprocessing_s": round(oprep, 3), "batch_queries_per_s": round(C2_BATCHES / oon, 1),
                               "cores": 1, "kind": "port",
                               "sample": f"the same DB, preprocessing and {C2_BATCHES} batches"}
    del g
    return out


# MS-MARCO-shaped private search (BASELINE.json metric's second dataset;
# reproduction/msmarco/reproduce.sh:224-230: private-search -n 3201821 -d 192
# -m 32 -k 100 -q 1000 -step 20 -parallel 3): synthetic d=192 vectors ~
# N(0, sigma_j), a degree-32 graph built on the GPU, k = 100,
# and every session runs past its 45-query maintenance window.
# 128 sessions in 4 teams (round 5, device loop): 8.65K q/s vs 7.2K for 64 in 2
# (tools/sweep_msmarco.sh, profiles/r05/ab/msmarco_sessions.log; 192 in 4: 8.97K)
MS_N, MS_DIM, MS_K, MS_SESSIONS, MS_GROUPS, MS_QUERIES, MS_WARMUP = 3_201_821, 192, 100, 128, 4, 48, 2


def private_search_msmarco(local, args, with_cpu: bool):
    import gc

    import pacmann_amd as pm
    from pacmann_amd.report import compute_recall
    from pacmann_amd.synth import msmarco_like_vectors
    ctx = pm.Context(local)
    v = msmarco_like_vectors(MS_N, MS_DIM, seed=501)
    ctx.sync()
    t0 = time.perf_counter()
    g, tm = pm.build_graph(v, M, 1.2, seed=502, ctx=ctx)
    build = {k: round(x, 4) for k, x in tm.items()}
    build["total_s"] = round(time.perf_counter() - t0, 4)
    # queries: warm-up, the timed region, then the kernel-timing pass's own
    S2, nq = args.ms_sessions or MS_SESSIONS, MS_WARMUP + 2 * MS_QUERIES
    ms_groups = args.ms_groups or MS_GROUPS
    rng = np.random.default_rng(503)
    qs = (v[rng.integers(0, MS_N, S2 * nq)] + rng.normal(0, 0.1, (S2 * nq, MS_DIM))).astype(np.float32)
    qs = qs.reshape(S2, nq, MS_DIM)
    base = pm.PIRGraphInfo(v, g, pir_seed=601, search_seed=602, ctx=ctx)
    base.Preprocess()
    sess = [base] + [base.Session(601 + i, 602 + i, pm.Context(local)) for i in range(1, S2)]
    for s_ in sess[1:]:
        s_.Preprocess()
    ctxs = [s_.ctx for s_ in sess]
    pm.search_loop_batched(sess, qs[:, :MS_WARMUP], MS_K, STEP, PARALLEL, ms_groups, args.threads)
    for c in ctxs:
        c.sync()
    # the timed region runs uninstrumented (as the headline's); the kernels are
    # timed over a second region of fresh queries (events in every dispatch
    # packet cost the rate a few per cent)
    q1 = MS_WARMUP + MS_QUERIES
    t0 = time.perf_counter()
    ans, _, online, maint = pm.search_loop_batched(sess, qs[:, MS_WARMUP:q1], MS_K, STEP, PARALLEL, ms_groups,
                                                   args.threads)
    for c in ctxs:
        c.sync()
    wall = time.perf_counter() - t0
    preps = [s_.PIR.stats()["PrepCount"] for s_ in sess]
    for c in ctxs:
        c.timing_reset()
        c.timing(2)
    t0 = time.perf_counter()
    pm.search_loop_batched(sess, qs[:, q1:], MS_K, STEP, PARALLEL, ms_groups, args.threads)
    for c in ctxs:
        c.sync()
    wall_kt = time.perf_counter() - t0
    for c in ctxs:
        c.timing(False)

    def tsum(name):
        r = [c.timing_get(name) for c in ctxs]
        return tuple(sum(x[i] for x in r) for i in range(3))
    kt = {k: tsum(k) for k in ("prep_offsets", "prep_fold", "prep_repl", "hint_match", "resolve", "match_resolve",
                                "answer")}
    tq = qs[:, MS_WARMUP:q1].reshape(-1, MS_DIM)
    gt = pm.knn(v, tq, K_TOP, ctx)
    recall = compute_recall(gt, ans.reshape(-1, MS_K)[:, :K_TOP], K_TOP)
    out = {"workload": "MS-MARCO-shaped private search (reproduce.sh:224-230): 3,201,821 x d=192 synthetic "
                       "vectors (16-d latent mixture, per-dimension sigma 0.82 -> 0.29 as the reference's PCA "
                       "fixture), degree-32 graph built on the GPU, 896-B PIR entries "
                       "(16 partitions, CS 1,024 / SS 196), k = 100, step 20, parallel 3",
           "sessions": S2, "lockstep_groups": ms_groups, "queries_per_session": MS_QUERIES,
           "private_queries_per_s": round(S2 * MS_QUERIES / wall, 2), "wall_s": round(wall, 4),
           "online_s_per_query": round(float(np.mean(online)) / MS_QUERIES, 6),
           "maintenance_s_per_query": round(float(np.mean(maint)) / MS_QUERIES, 6),
           "maintenances_in_region": int(sum(preps) - S2),   # PrepCount is 1 after the first preprocessing
           "recall_at_10": round(float(recall), 4), "graph_build": build,
           "kernel_timing_pass": {"queries_per_session": MS_QUERIES, "wall_s": round(wall_kt, 4),
                                  "private_queries_per_s": round(S2 * MS_QUERIES / wall_kt, 2)},
           "kernel_avg_us": {k: round(x[1] / x[0] * 1e3, 3) for k, x in kt.items() if x[0]}}
    n, ms, by = kt["answer"]
    if n and by:
        ach = (by / n) / (ms / n / 1e3) / 1e9
        out["roofline"] = {"bound": "hbm", "kernel": "answer", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "avg_ms": round(ms / n, 5),
                           "launches": n, "alg_bytes_per_launch": by / n,
                           "aggregate": {"achieved": round(by / wall_kt / 1e9, 1),
                                         "frac": round(by / wall_kt / 1e9 / HBM_PEAK_GBS, 4)}}
        attach_traffic(out["roofline"], SYMBOLS["answer"], answer_grid((S2 // ms_groups) * PARALLEL * M))
    n, ms, by = kt["prep_fold"]
    if n and by:   # the maintenance fold's entry reads against the LDS ds_read_b128 aggregate
        ach = (by / n) / (ms / n / 1e3) / 1e9
        out["roofline_prep"] = {"bound": "lds", "kernel": "prep_fold", "achieved": round(ach, 1),
                                "peak": LDS_B128_PEAK_GBS, "unit": "GB/s", "frac": round(ach / LDS_B128_PEAK_GBS, 4),
                                "avg_ms": round(ms / n, 3), "launches": n, "alg_bytes_per_launch": by / n}
    if "roofline" in out:   # the whole private query against its three ceilings
        out["roofline"]["composite"] = composite_floor(kt, S2, MS_QUERIES, base.PIR, out["private_queries_per_s"],
                                                       ss_r2=base.PIR.SubConfig(0)["SetSize"],
                                                       entry_words=(MS_DIM + M) // 2)
    if with_cpu:   # the oracle replaying session 0's workload, one core
        cb = cpu_baseline(v, g, qs[0, :q1], MS_WARMUP, ans[0], ctx, 601, 602, k=MS_K)
        out["cpu_baseline"] = cb
    del sess, base, ctxs
    gc.collect()
    return out


# BASELINE.json configs[3] / configs[4]: private graph search over a sharded
# BIGANN-scale graph DB.  No 10^8 / 10^9-vector dataset or graph can be built
# or shipped here, so the graph is the reference's synthetic mode
# (private-search.go:42-69,114-117,168-170: uniform [0,1) f32 vectors, uniform
# neighbour ids, uniform [0,1) queries) generated on the device from a seed
# (pm_graph_create_synth); entries are PIRGraphInfo's d = 128, m = 32 wire
# format, (128 + 32) * 4 B = 640 B = 80 words.  S client sessions per GPU run
# the full private-search.go loop (SearchKNN over PIRGraphInfo, 20 rounds of
# 96 ids, maintenance trigger) in lock-step teams over this rank's shard of the
# batch PIR (partitions p % layout == shard); every shared step ends in ONE
# combine of the team's per-id records (RCCL all-reduce over xGMI when the
# layout is spread over the job's ranks).  A layout wider than the job (the
# 1B DB on fewer than 8 GPUs: 640 GB does not fit one GPU's 288 GB) runs one
# shard per GPU with the other shards' answers generated from the graph's
# spec on the device (modelled peers: their PIR work is not measured).
BIG_DIM, BIG_E, BIG_SEARCH_Q, BIG_SEARCH_WARMUP, BIG_GROUPS = 128, 80, 36, 2, 2   # 36 queries: a ~0.3 s timed region (12 gave ~0.09 s, +-20 % between boxes)
BIG_SESSIONS = {"config3_bigann_100m": 32, "config4_bigann_1b": 16}   # caps; memory decides below


def client_bytes(sub: dict, E: int) -> int:
    """Device bytes of one client's state for one partition (engine_create's
    arrays: tags, program points, parities, replacement rows, histogram,
    local cache arena, the tag-major PRF table tabT and the search row cur;
    the chunk-major table tab is not allocated for the BIGANN shapes, whose
    fold reads tabT: pmk::fold_needs_tab)."""
    PH, SS, Q, MQ = sub["PrimaryHintNum"], sub["SetSize"], sub["MaxQueryPerChunk"], sub["MaxQueryNum"]
    H = PH + SS * Q
    return (H * 4 + PH * 4 + H * E * 8 + SS * Q * (4 + E * 8) + SS * 4 + MQ * E * 8
            + (SS + 7) // 8 * 8 * H * 2 + PH * SS * 2)


def bigann_layout(key: str, ws: int, rank: int) -> dict:
    """Rank -> shard mapping of the BIGANN blocks.  configs[3] names BIGANN-100M
    "sharded across 4 MI355X": with 4 or 8 ranks it is served as 4-rank layouts
    (ws / 4 replicas, each a 4-way shard of the same DB with its own sessions;
    no collective between replicas), with 1-3 ranks as one layout over all of
    them.  configs[4] is the 8-way layout of BIGANN-1B: below 8 ranks each rank
    serves one shard and the other shards' answers are modelled."""
    if key == "config3_bigann_100m":
        layout = 4 if ws >= 4 and ws % 4 == 0 else ws
    else:
        layout = 8
    replicas = max(1, ws // layout) if layout <= ws else 1
    replica = rank // layout if layout <= ws else 0
    modelled = layout > ws
    combine = layout <= ws and layout > 1
    return {"layout": layout, "shard": rank % layout, "replica": replica, "replicas": replicas,
            "modelled": modelled, "combine": combine,
            "group_ranks": [replica * layout + i for i in range(layout)] if combine else [rank]}


def replica_groups(dist, ws: int, layout: int):
    """One gloo group per replica of a layout (ranks r*layout .. r*layout +
    layout - 1), created by every rank in the same order (new_group is
    collective); the replica's combine agrees and falls back inside it."""
    return [dist.new_group(list(range(r * layout, (r + 1) * layout)), backend="gloo") for r in range(ws // layout)]


def bigann_rates(replicas: int, S: int, Q: int, elapsed: float, maint_in_region_s: float, prep_client_s: float,
                 support: int) -> dict:
    """The reference metric (private-search.go:216-240: queries / (online +
    maintenance), maintenance at the harness's cadence) for a block whose timed
    region is shorter than one maintenance window: the region's online wall
    time plus every session's re-preprocessing amortised over its window of
    SupportBatchNum / (step x parallel) queries (a client's preprocessing time,
    measured in the block; the S clients' preprocessings run one after another
    on the GPU).  value counts every replica's sessions."""
    window = support / (STEP * PARALLEL)
    online = max(1e-9, elapsed - maint_in_region_s)
    cadence = online + Q * S * prep_client_s / window
    return {"private_queries_per_s": round(replicas * S * Q / elapsed, 2),
            "private_queries_per_s_at_maintenance_cadence": round(replicas * S * Q / cadence, 2),
            "private_queries_per_s_online_only": round(replicas * S * Q / online, 2),
            "maintenance_window_queries": round(window, 2)}


def bigann_search(key, name, n_entries, lay, rank, ws, local, dist, comb_group, args, nccl_group_fn=None,
                  replica_group=None):
    """comb_group: the preferred combine when the layout spans the ranks
    ("native" RCCL inside the library, "torch-rccl" or "gloo"); nccl_group_fn()
    gives the torch RCCL group (probed and agreed) or None."""
    import gc

    import torch

    import pacmann_amd as pm
    from pacmann_amd.shard import RecordCombiner
    layout, shard, modelled, combine = lay["layout"], lay["shard"], lay["modelled"], lay["combine"]
    replica, replicas = lay["replica"], lay["replicas"]
    rs = 1000 * replica   # each replica serves its own sessions and queries
    progress(f"  {key}: shard {shard} of {layout}, replica {replica} of {replicas}" +
             (" (other shards modelled)" if modelled else ""))
    ctx = pm.Context(local)
    ctx.timing(1)
    t0 = time.perf_counter()
    base = pm.PIRGraphInfo.Synthetic(n_entries, BIG_DIM, M, data_seed=51, shard=shard, nshards=layout,
                                     pir_seed=61 + rs, search_seed=62 + rs, ctx=ctx)
    base.Preprocess()   # the DB generated on the device, then the first client's preprocessing
    ctx.sync()
    t_base = time.perf_counter() - t0
    ctx.timing(False)
    kprep = {k: ctx.timing_get(k) for k in ("prep_offsets", "prep_fold", "prep_repl")}
    pir = base.PIR
    stats = pir.stats()
    own = [p for p in range(stats["PartitionNum"]) if p % layout == shard]
    subs = [pir.SubConfig(p) for p in own]
    per_client = sum(client_bytes(c, BIG_E) for c in subs)
    free, _ = ctx.mem_info()
    S = int(max(1, min(BIG_SESSIONS[key], 1 + (free * 0.8) // per_client)))
    if args.big_sessions:
        S = min(S, args.big_sessions)
    if dist:   # the same sessions on every rank
        t = torch.tensor([S], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        S = int(t.item())
    sess = [base] + [base.Session(61 + rs + i, 62 + rs + i, pm.Context(local)) for i in range(1, S)]
    for x in sess[1:]:
        x.Preprocess()
    ctxs = [x.ctx for x in sess]
    nq = BIG_SEARCH_WARMUP + 2 * BIG_SEARCH_Q   # warm-up, the timed region, the kernel-timing pass
    qs = np.random.default_rng(63 + rs).random((S, nq, BIG_DIM), dtype=np.float32)   # genRandomMatrix queries
    groups = min(args.big_groups or BIG_GROUPS, S)
    comb, comb_path, comb_note = None, None, None
    if combine:   # agreed by every rank, bounded, with fallbacks (shard.combiner_with_fallback)
        from pacmann_amd.shard import combiner_with_fallback
        words = [int(pm.lib().pm_sharded_record_words(sess[0].h, n, PARALLEL)) for n in pm.team_sizes(S, groups)]
        comb, comb_path, comb_note = combiner_with_fallback(words, local, prefer=comb_group,
                                                            nccl_group_fn=nccl_group_fn if replicas == 1 else None,
                                                            gloo_group=replica_group)
        progress(f"  {key}: combine path {comb_path}" + (f" ({comb_note})" if comb_note else ""))
    # the warm-up queries with every record checked on the host (pm_set_option
    # "verify_records": answered records against the graph's spec and the
    # reference-order L2, unanswered ids against their explanation); off in the
    # timed region
    for c in ctxs:
        c.timing_reset()
    pm.set_option("verify_records", 1)
    try:
        pm.search_loop_sharded(sess, qs[:, :BIG_SEARCH_WARMUP], K_TOP, STEP, PARALLEL, groups, args.threads,
                               combiner=comb, model_peers=modelled)
    finally:
        pm.set_option("verify_records", 0)
    recs = {k: sum(c.timing_get("host_records_" + k)[0] for c in ctxs)
            for k in ("verified", "bad", "dropped", "failed", "peer", "unexplained")}
    def tsum(name):
        r = [c.timing_get(name) for c in ctxs]
        return tuple(sum(x[i] for x in r) for i in range(3))

    # the timed region runs uninstrumented (host timers only); the kernels are
    # timed over a second region of fresh queries, run by every rank alike
    q1 = BIG_SEARCH_WARMUP + BIG_SEARCH_Q
    for c in ctxs:
        c.sync()
        c.timing_reset()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ans, wall, online, maint = pm.search_loop_sharded(sess, qs[:, BIG_SEARCH_WARMUP:q1], K_TOP, STEP, PARALLEL,
                                                      groups, args.threads, combiner=comb, model_peers=modelled)
    for c in ctxs:
        c.sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ht = {k: tsum(k) for k in ("host_combine", "host_combine_turn", "host_step_wait", "host_batch_query",
                                "host_gvi_parse", "host_step_launch", "host_step_post", "host_knn_update",
                                "host_knn_batch", "host_knn_init")}
    for c in ctxs:
        c.timing_reset()
        c.timing(2)
    t0 = time.perf_counter()
    pm.search_loop_sharded(sess, qs[:, q1:], K_TOP, STEP, PARALLEL, groups, args.threads, combiner=comb,
                           model_peers=modelled)
    for c in ctxs:
        c.sync()
    if dist:
        dist.barrier()
    elapsed_kt = time.perf_counter() - t0
    for c in ctxs:
        c.timing(False)
    kt = {k: tsum(k) for k in ("hint_match", "resolve", "match_resolve", "gather", "answer", "pack_records",
                                "synth_records", "combine", "prep_offsets", "prep_fold", "prep_repl", "l2_rows")}
    combine_paths = None
    if key == "config3_bigann_100m" and ws == 1 and not args.no_combine_probe:
        combine_paths = combine_probe(sess, qs, groups, args, local)
    rounds = BIG_SEARCH_Q * STEP * groups   # shared steps in the timed region (every team)
    same = None if modelled else 1   # modelled layouts: each rank serves another shard (its own failures)
    if dist and not modelled:   # every rank holds the same answers (the combined records drive identical searches)
        h = torch.tensor([int(np.bitwise_xor.reduce(ans.ravel().astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)))
                          & ((1 << 62) - 1)], dtype=torch.int64)
        hmax, hmin = h.clone(), h.clone()
        dist.all_reduce(hmax, op=dist.ReduceOp.MAX, group=replica_group)   # the ranks of this layout
        dist.all_reduce(hmin, op=dist.ReduceOp.MIN, group=replica_group)
        same = int(hmax.item() == hmin.item())
    if dist:
        t = torch.tensor([elapsed, t_base], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, t_base = (float(x) for x in t)
    tot, succ = 0, 0
    for x in sess:
        a, b = x.counts()
        tot, succ = tot + a, succ + b
    prep_client = kprep["prep_offsets"][1] + kprep["prep_fold"][1] + kprep["prep_repl"][1]   # one client, ms

    def roof(entry, nbytes=None):
        n, ms, by = entry
        by = nbytes if nbytes is not None else by
        if not n or not ms or not by:
            return None
        ach = (by / n) / (ms / n / 1e3) / 1e9
        return {"avg_ms": round(ms / n, 5), "launches": n, "alg_bytes_per_launch": by / n, "achieved": round(ach, 1),
                "unit": "GB/s", "peak": HBM_PEAK_GBS, "frac": round(ach / HBM_PEAK_GBS, 4)}
    fold = roof(kprep["prep_fold"])
    if fold:
        rows_local = sum(c["DBSize"] for c in subs)
        comp = rows_local * BIG_E * 8
        fold["compulsory"] = {"bytes": comp, "achieved": round(comp / (fold["avg_ms"] / 1e3) / 1e9, 1),
                              "frac": round(comp / (fold["avg_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS, 4)}
    gkey = "gather" if kt["gather"][0] else "answer"
    ans_roof = roof(kt[gkey])
    if ans_roof:
        ans_roof["kernel"] = gkey
    support = stats["SupportBatchNum"]
    maint_model = prep_client / 1e3 / support * STEP * PARALLEL   # one client's amortised maintenance (:298)
    n_comb, ms_comb, by_comb = kt["combine"]
    out = {
        "workload": f"{name}, {layout}-way layout" + (f" x {replicas} replicas" if replicas > 1 else "") +
                    f": private graph search (SearchKNN over PIRGraphInfo, k = {K_TOP}, step {STEP}, "
                    f"parallel {PARALLEL}) over a {n_entries:,}-vertex synthetic graph (the reference's -input "
                    f"synthetic mode: uniform [0,1) d = {BIG_DIM} vectors, uniform degree-{M} neighbours, uniform "
                    f"queries) generated on the device; 640-B entries, BatchSize 32 (16 partitions), "
                    f"FailureProbLog2 8",
        "n_ranks": ws, "layout_shards": layout, "shard": shard, "replicas": replicas, "replica": replica,
        "peers": ("modelled: the other shards' answers generated from the graph's spec on the device "
                  f"({layout} shards, {ws} GPU(s); their PIR work is not measured)" if modelled else
                  "RCCL all-reduce of the team's records per shared step, inside libpacmann.so (pm_rccl_combine)"
                  if comb_path == "native" else
                  "RCCL all-reduce of the team's records per shared step (torch.distributed callback)"
                  if comb_path == "torch-rccl" else
                  "gloo all-reduce of the team's records per shared step" if comb_path == "gloo" else
                  "none (one rank holds every partition)"),
        "combine_path": comb_path, "combine_fallback": comb_note,
        "sessions": S, "sessions_per_replica": S, "lockstep_groups": groups, "queries_per_session": BIG_SEARCH_Q,
        **bigann_rates(replicas, S, BIG_SEARCH_Q, elapsed, float(np.max(maint)), prep_client / 1e3, support),
        "cadence_note": "private_queries_per_s is the timed region's rate (every replica's sessions; the region "
                        "is shorter than one maintenance window, so it holds no re-preprocessing); "
                        "_at_maintenance_cadence is the reference's metric (private-search.go:216-240): the "
                        "region's online time plus each session's re-preprocessing (the one-client "
                        "preprocessing measured in this block, clients one after another) amortised over its "
                        "window; quote that one",
        "wall_s": round(elapsed, 4),
        "kernel_timing_pass": {"queries_per_session": BIG_SEARCH_Q, "wall_s": round(elapsed_kt, 4),
                               "note": "a second region of fresh queries with every kernel's events on; the "
                                       "kernel averages and rooflines below come from it"},
        "ms_per_round": round(elapsed / (BIG_SEARCH_Q * STEP) * 1e3, 4),
        "online_s_per_query": round(float(np.mean(online)) / BIG_SEARCH_Q, 6),
        "maintenance_s_per_query_in_region": round(float(np.mean(maint)) / BIG_SEARCH_Q, 6),
        "maintenance_s_per_query_amortised": round(maint_model, 6),
        "support_batch_num": support, "partitions_per_rank": len(own),
        "rank_db_gb": round(sum(c["DBSize"] for c in subs) * BIG_E * 8 / 1e9, 2),
        "client_state_gb": round(per_client / 1e9, 2),
        "subconfig": {k: subs[0][k] for k in ("ChunkSize", "SetSize", "PrimaryHintNum", "MaxQueryPerChunk",
                                              "MaxQueryNum")},
        "db_and_first_client_s": round(t_base, 3), "preprocessing_ms_one_client": round(prep_client, 3),
        "kernel_avg_us": {k: round(v[1] / v[0] * 1e3, 3) for k, v in {**kt, **kprep}.items() if v[0]},
        "combine": {"launches": n_comb, "ms_per_round": round(ms_comb / n_comb, 5) if n_comb else None,
                    "bytes_per_round": by_comb / n_comb if n_comb else 0,
                    "host_ms_per_round": round(ht["host_combine"][1] / max(1, ht["host_combine"][0]), 5),
                    "turn_wait_ms_per_round": round(ht["host_combine_turn"][1] / max(1, ht["host_combine_turn"][0]), 5),
                    "note": "device time of the in-place all-reduce on the team stream (events around the "
                            "combine), per shared step; host_ms is the callback's wall time"},
        "host_ms_per_round": {k[5:]: round(v[1] / (BIG_SEARCH_Q * STEP), 4) for k, v in ht.items() if v[1]},
        "combine_paths_world1": combine_paths,
        "pir_scan_fold": fold, "pir_scan_answer": ans_roof,
        "roofline_prf": prf_roofline(kprep["prep_offsets"], "k_prep_offsets of one client's preprocessing",
                                     subs[0]["SetSize"]),
        "check": {"ids_fetched": tot, "ids_answered": succ, "ranks_identical": None if same is None else bool(same),
                  "records_checked_in_warmup": recs,
                  "note": "warm-up rounds: every answered record equal to the graph's row (synthetic spec) and the "
                          "reference-order L2 (verified) or not (bad); unanswered ids explained by the overflow "
                          "drop (batch-pir.go:195-200), a failed sub-query of this rank, or another rank's"},
    }
    del sess, base, ctxs, pir
    gc.collect()
    ctx.close()
    return out


# BASELINE.json configs[0]: graphann_test.go's InnerProduct benchmark
# (graphann_test.go:221-284): N = 1e8 rows of D = 128 uint32, v[i*D+j] = i+j,
# q[j] = j, the sum of all row products mod 2^32 (closed form 1,178,525,696).
C0_N, C0_D, C0_SUM, C0_CPU_ROWS = 100_000_000, 128, 1_178_525_696, 1 << 23
IP_SCAN_SYMBOL = ("pm::k_ip_scan(HIP_vector_type<unsigned int, 4u> const*, unsigned long, unsigned int const*, "
                  "unsigned int, unsigned int*)")   # as rocprofv3 names it
IP_SCAN_GRID = 2048 * 256   # pmk::ip_rows' scan launch: 2,048 workgroups of 256 threads (pm_kernels.hip)


def inner_product_scan(ctx, with_cpu: bool):
    """The scan on the GPU (51.2 GB filled on the device, then one streaming
    k_ip_scan launch timed with events on its stream; mean of 3), against HBM
    peak; the oracle's AVX-512-equivalent InnerProduct over a materialised
    sample of the same rows on 1 and on all host cores beside it."""
    import pacmann_amd as pm
    runs = [pm.ip_bench(C0_N, C0_D, ctx) for _ in range(3)]
    ok = all(s == C0_SUM for s, _ in runs)
    ms = sum(m for _, m in runs) / len(runs)   # the mean, like rocprof's average over the same launches
    nbytes = C0_N * C0_D * 4
    ach = nbytes / (ms / 1e3) / 1e9
    out = {"workload": "graphann_test.go InnerProduct bench (configs[0]): 1e8 x 128 uint32 rows v[i*D+j]=i+j, "
                       "q[j]=j, sum mod 2^32",
           "sum_ok": ok, "scan_ms": round(ms, 4), "rows_per_s": round(C0_N / (ms / 1e3), 1),
           "roofline": {"bound": "hbm", "kernel": "ip_scan", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": nbytes,
                        "avg_ms": round(ms, 5), "launches": len(runs)}}
    attach_traffic(out["roofline"], IP_SCAN_SYMBOL, IP_SCAN_GRID)
    if with_cpu:
        from oracle import oracle as O
        rows = np.arange(C0_CPU_ROWS, dtype=np.uint32)[:, None] + np.arange(C0_D, dtype=np.uint32)[None, :]
        q = np.arange(C0_D, dtype=np.uint32)
        ncores = min(16, os.cpu_count() or 1)   # the box's CPU share is 16 cores per GPU
        cpu = {}
        for th in (1, ncores):
            t0 = time.perf_counter()
            O.inner_product_scan(rows, q, th)
            dt = time.perf_counter() - t0
            cpu[th] = rows.nbytes / dt / 1e9
        del rows
        out["cpu_baseline"] = {"value": round(cpu[1], 2), "unit": "GB/s", "cores": 1, "kind": "port",
                               "all_cores": {"value": round(cpu[ncores], 2), "cores": ncores},
                               "sample": f"{C0_CPU_ROWS:,} materialised rows (4.3 GB) of the same fill"}
    return out


def ip_shard_rows(n, ws, rank):
    """Rows [r0, r1) of the InnerProduct fill scanned by `rank` of `ws`
    (the scan shards by rows)."""
    return n * rank // ws, n * (rank + 1) // ws


def ip_closed_form(r0, r1, d):
    """sum_{r0 <= i < r1, j < d} (i + j) * j mod 2^32 (graphann_test.go:249-283's
    fill v[i*D+j] = i+j, q[j] = j): rows [0, 1e8) at D = 128 give 1,178,525,696."""
    n = r1 - r0
    return ((r0 + r1 - 1) * n // 2 * (d * (d - 1) // 2) + n * ((d - 1) * d * (2 * d - 1) // 6)) % (1 << 32)


def inner_product_scan_sharded(ctx, dist, rank, ws, local, nccl_group_fn):
    """configs[0] over the job's ranks: rank r scans its rows of the 1e8-row
    fill (ip_shard_rows; the same kernel, timed the same way, mean of 3), the
    ranks' mod-2^32 sums are added by one all-reduce (over RCCL when the
    agreed RCCL group exists, else gloo) and checked against the closed form;
    scan time = the slowest rank's.  Total work fixed: strong scaling."""
    import torch

    import pacmann_amd as pm
    r0, r1 = ip_shard_rows(C0_N, ws, rank)
    runs = [pm.ip_bench(C0_N, C0_D, ctx, r0=r0, rows=r1 - r0) for _ in range(3)]
    mine_ok = all(sm == ip_closed_form(r0, r1, C0_D) for sm, _ in runs)
    ms_local = sum(m for _, m in runs) / len(runs)
    grp = nccl_group_fn() if nccl_group_fn else None
    sums = torch.tensor([sm for sm, _ in runs], dtype=torch.int64)
    if grp is not None:   # the partial sums through RCCL (xGMI), like the reference's total
        t = sums.to(f"cuda:{local}")
        dist.all_reduce(t, group=grp)
        total = t.cpu()
    else:
        dist.all_reduce(sums)
        total = sums
    ok = all((int(x) & 0xFFFFFFFF) == C0_SUM for x in total)
    agg = torch.tensor([ms_local, float(mine_ok)], dtype=torch.float64)
    mx, mn = agg.clone(), agg.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(mn, op=dist.ReduceOp.MIN)
    ms = float(mx[0])
    nbytes = (r1 - r0) * C0_D * 4
    ach = nbytes / (ms_local / 1e3) / 1e9
    out = {"workload": "graphann_test.go InnerProduct bench (configs[0]): 1e8 x 128 uint32 rows v[i*D+j]=i+j, "
                       f"q[j]=j, sum mod 2^32, rows sharded over {ws} GPUs",
           "n_ranks": ws, "scaling": "strong", "shard_rows": r1 - r0,
           "collective": "rccl" if grp is not None else "gloo",
           "sum_ok": ok, "shard_sums_ok": bool(mn[1] == 1.0),
           "scan_ms": round(ms, 4), "rows_per_s": round(C0_N / (ms / 1e3), 1),
           "roofline": {"bound": "hbm", "kernel": "ip_scan", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "alg_bytes_per_launch": nbytes,
                        "avg_ms": round(ms_local, 5), "launches": len(runs),
                        "note": "rank 0's shard; scan_ms above is the slowest rank's"}}
    return out


def combine_probe(sess, qs, groups, args, local):
    """World 1: the sharded loop's two combine paths over a one-rank job, a
    few queries each on the block's sessions (results not in the block's
    numbers): the torch.distributed callback over an RCCL group
    (RecordCombiner) and the library-native RCCL communicators
    (pm_rccl_combine).  Per shared step: the device time of the all-reduce on
    the team stream and the host wall time of the combine call."""
    import datetime
    import socket

    import torch
    import torch.distributed as dist

    import pacmann_amd as pm
    from pacmann_amd.shard import RcclCombiner, RecordCombiner
    out = {}
    try:
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                timeout=datetime.timedelta(seconds=120))
        torch.cuda.set_device(local)
        ng = dist.new_group(backend="nccl")
        ctxs = [x.ctx for x in sess]
        nq = 2
        for name, comb in (("torch_callback", RecordCombiner(group=ng, device=local)),
                           ("native", RcclCombiner(group=None, device=local))):
            pm.search_loop_sharded(sess, qs[:, :1], K_TOP, STEP, PARALLEL, groups, args.threads, combiner=comb)
            for c in ctxs:
                c.sync()
                c.timing_reset()
                c.timing(1)
            t0 = time.perf_counter()
            pm.search_loop_sharded(sess, qs[:, 1:1 + nq], K_TOP, STEP, PARALLEL, groups, args.threads, combiner=comb)
            for c in ctxs:
                c.sync()
            wall = time.perf_counter() - t0
            for c in ctxs:
                c.timing(False)
            n, ms, _ = (sum(x) for x in zip(*[c.timing_get("combine") for c in ctxs]))
            hn, hms, _ = (sum(x) for x in zip(*[c.timing_get("host_combine") for c in ctxs]))
            out[name] = {"rounds": int(hn), "device_ms_per_round": round(ms / n, 5) if n else None,
                         "host_ms_per_round": round(hms / hn, 5) if hn else None,
                         "private_queries_per_s": round(len(sess) * nq / wall, 2)}
            if name == "native":
                comb.close()
        out["note"] = ("one-rank job: the all-reduce moves nothing between GPUs; the host time is the per-step "
                       "cost of issuing it (torch callback: ctypes -> GIL -> ProcessGroupNCCL; native: one "
                       "ncclAllReduce call inside libpacmann.so)")
    except Exception as e:   # recorded, never fatal
        out["error"] = f"{type(e).__name__}: {e}"
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    return out


def dist_init():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws == 1:
        return None, 0, 1, 0
    import datetime

    import torch.distributed as dist
    # control plane (barrier, max of timings) over gloo; bounded so a lost rank
    # ends the run instead of hanging it
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=600))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    ndev = torch.cuda.device_count()   # counting devices does not initialise HIP
    # more ranks than GPUs (a rehearsal on one GPU): ranks share devices round-robin
    return dist, dist.get_rank(), ws, local % max(ndev, 1)


def prf_roofline(entry, note, set_size=None):
    """AES-PRF throughput of k_prep_offsets launches (timing entry: launches,
    ms, PRFs evaluated) against the T-table lookup ceiling of the form that
    ran (SetSize <= 256: round 2 hoisted, 112 lookups per PRF; else 122.5)."""
    n, ms, prfs = entry
    if not n or not ms or not prfs:
        return None
    lk = AES_LOOKUPS_PER_PRF_R2 if set_size is not None and set_size <= 256 else AES_LOOKUPS_PER_PRF
    peak = prf_peak_g(lk)
    g = prfs / (ms / 1e3) / 1e9
    return {"bound": "lds", "kernel": "prep_offsets", "achieved": round(g, 2), "peak": round(peak, 2),
            "unit": "G PRF/s", "frac": round(g / peak, 4), "launches": n, "avg_ms": round(ms / n, 5),
            "prfs_per_launch": prfs / n, "lookups_per_prf": lk,
            "note": f"{note}: AES-128 blocks per second against the conflict-free ds_read_b32 lookup rate "
                    f"(~75 TB/s = 18.75 T lookups/s) / {lk} lookups per PRF (pm_aes.h); the "
                    "~2 VALU per lookup put the vector-issue ceiling at about the same rate"}


def composite_floor(ktime, S, queries_per_session, pir, value_per_gpu, ss_r2=None, entry_words=(DIM + M) // 2):
    """The whole private query's GPU floor: per session
    query, its answer bytes at HBM peak + its share of the maintenance fold's
    entry reads at the LDS ds_read_b128 aggregate + its share of the PRFs at the
    AES T-table ceiling, the shares over the harness's actual maintenance
    cadence (private-search.go:226-232: FinishedBatchNum + step*parallel + 10 >=
    SupportBatchNum, FinishedBatchNum advancing step*(parallel*m/BatchSize) per
    query).  `frac` = value per GPU / the floor's q/s.  From the kernel-timing
    pass, which holds one maintenance of every session."""
    na, _, ab = ktime["answer"]
    nf, _, fb = ktime["prep_fold"]
    npf, _, prfs = ktime["prep_offsets"]
    if not (na and ab and nf and fb and npf and prfs):
        return None
    st = pir.stats()
    fbn_per_q = STEP * (PARALLEL * M // st["BatchSize"])
    cadence = -(-(st["SupportBatchNum"] - STEP * PARALLEL - 10) // fbn_per_q)   # queries between maintenances
    clients = max(1, round(fb / sum(((c["PrimaryHintNum"] + (c["SetSize"] - 1) * c["MaxQueryPerChunk"]) * c["SetSize"]
                                      * entry_words * 8)
                                     for c in (pir.SubConfig(p) for p in range(st["PartitionNum"])))))
    ans_q = ab / (S * queries_per_session)
    fold_q = fb / clients / cadence
    prf_q = prfs / clients / cadence
    lk = AES_LOOKUPS_PER_PRF_R2 if ss_r2 is not None and ss_r2 <= 256 else AES_LOOKUPS_PER_PRF
    t_ans = ans_q / (HBM_PEAK_GBS * 1e9)
    t_fold = fold_q / (LDS_B128_PEAK_GBS * 1e9)
    t_prf = prf_q / (prf_peak_g(lk) * 1e9)
    floor = t_ans + t_fold + t_prf
    return {"unit": "us per private query", "answer_us": round(t_ans * 1e6, 3), "fold_us": round(t_fold * 1e6, 3),
            "prf_us": round(t_prf * 1e6, 3), "floor_us": round(floor * 1e6, 3),
            "floor_queries_per_s": round(1 / floor, 1), "frac": round(value_per_gpu * floor, 4),
            "maintenance_cadence_queries": cadence, "clients_per_maintenance": clients,
            "per_query": {"answer_bytes": ans_q, "fold_bytes": fold_q, "prfs": prf_q},
            "note": "answer bytes at HBM peak + the fold's entry reads at the LDS ds_read_b128 aggregate + the "
                    "PRFs at the T-table lookup ceiling, per private query (maintenance amortised over its actual "
                    "cadence); frac = value per GPU x floor"}


def read_timeline(path):
    """Per kernel of a pm_timing_timeline file: launches, summed and union
    milliseconds; "query_phase": the span before the first maintenance kernel
    and the share of it with any kernel running."""
    rows = []
    with open(path) as f:
        for ln in f:
            n, a, b, _ = ln.strip().split(",")
            rows.append((float(a), float(b), n))
    if not rows:
        return {}

    def union(iv):
        tot, cs, ce = 0.0, None, None
        for a, b in sorted(iv):
            if ce is None or a > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        return tot + (ce - cs if ce is not None else 0.0)

    out = {}
    for n in sorted({r[2] for r in rows}):
        iv = [(a, b) for a, b, m in rows if m == n]
        out[n] = {"launches": len(iv), "sum_ms": round(sum(b - a for a, b in iv) / 1e3, 3),
                  "union_ms": round(union(iv) / 1e3, 3)}
    t0 = min(r[0] for r in rows)
    prep = [a for a, b, n in rows if n.startswith("prep_")]
    if prep:
        t1 = min(prep)
        q = [(a, min(b, t1)) for a, b, n in rows if a < t1]
        out["query_phase"] = {"ms": round((t1 - t0) / 1e3, 3),
                              "busy_frac": round(union(q) / max(t1 - t0, 1e-9), 4),
                              "note": "kernel-timing pass before its maintenance: share with any kernel running"}
    return out


def rccl_group(dist, local, out):
    """An RCCL (nccl backend) group over all ranks for the sharded blocks'
    combine, or None (the shards then combine over the gloo group).  RCCL
    creates its communicator at the first collective, so a one-element
    all-reduce runs inside the attempt; the ranks then agree over gloo (MIN of
    their success flags), so either every rank uses RCCL or none does."""
    import datetime

    import torch
    grp, ok = None, 1
    try:
        torch.cuda.set_device(local)
        grp = dist.new_group(backend="nccl", timeout=datetime.timedelta(seconds=180))
        t = torch.ones(1, device=f"cuda:{local}")
        dist.all_reduce(t, group=grp)
        torch.cuda.synchronize(local)
        ok = int(t.item() == dist.get_world_size())
        if not ok:
            out["rccl_group_error"] = f"probe all-reduce gave {t.item()}"
    except Exception as e:   # recorded; the shards then combine over the gloo group
        ok = 0
        out["rccl_group_error"] = f"{type(e).__name__}: {e}"
    flag = torch.tensor([ok], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)   # default (gloo) group: every rank decides alike
    if int(flag.item()) != 1:
        out.setdefault("rccl_group_error", "another rank could not use RCCL")
        return None
    return grp


class Watchdog:
    """Ends the run with the line written if the multi-rank blocks overrun
    `budget_s` (a peer stuck in a collective, a bounded init that still
    fails to return): rank 0 writes the one JSON line with the unfinished
    blocks marked, every rank exits.  fire() is called by the main thread when
    the blocks finished: False if the watchdog got there first."""

    def __init__(self, out, rank, line_fd, budget_s, keys=("config3_bigann_100m", "config4_bigann_1b")):
        import threading
        self.out, self.rank, self.line_fd, self.budget_s, self.keys = out, rank, line_fd, budget_s, tuple(keys)
        self.lock = threading.Lock()
        self.done = False
        self.timer = threading.Timer(budget_s, self._expire) if budget_s > 0 else None
        if self.timer:
            self.timer.daemon = True
            self.timer.start()

    def put(self, key, value):
        """The main thread's block results go into the line under the lock, so
        the watchdog's snapshot never sees the dict change under it."""
        with self.lock:
            self.out[key] = value

    def _expire(self):
        with self.lock:
            if self.done:
                return
            self.done = True
            snap = dict(self.out)   # the blocks finished so far (each value is complete)
        for key in self.keys:
            snap.setdefault(key, {"error": "unfinished: the run's multi-rank budget expired (watchdog)"})
        # the hang is reported in the line AND by the exit status (3): the
        # headline and single-GPU blocks in the line are complete and valid,
        # the process is not (a block never returned)
        snap["watchdog"] = {"fired": True, "budget_s": self.budget_s}
        if self.rank == 0:
            os.write(self.line_fd, (json.dumps(snap) + "\n").encode())
        progress("watchdog: multi-rank blocks over budget; line written with watchdog.fired, exiting 3")
        os._exit(3)

    def fire(self) -> bool:
        with self.lock:
            if self.done:
                return False
            self.done = True
        if self.timer:
            self.timer.cancel()
        return True


def start_watchdog(out, rank, line_fd, budget_s, keys=("config3_bigann_100m", "config4_bigann_1b")):
    return Watchdog(out, rank, line_fd, budget_s, keys)


def cpu_baseline(v, g, q0, warmup, answers0, ctx, pir_seed, search_seed, k=K_TOP):
    """The oracle (single-thread C++ restatement of the Go/AVX path; its hint
    fold on one thread like the reference's ThreadNum = 1) replaying session
    0's exact workload: same graph, same PIR and search seeds, the same
    warm-up queries and then the same timed queries q0[warmup:].  value =
    queries / (online + maintenance) over the replay; its answers are compared
    with session 0's timed answers one by one, and both recalls are computed
    on those identical queries."""
    import pacmann_amd as pm
    from oracle import oracle as O
    from pacmann_amd.report import compute_recall
    O.set_prep_threads(1)
    og = O.Graph(v, g, pir_seed=pir_seed, search_seed=search_seed)
    t0 = time.perf_counter()
    og.Preprocess()
    prep = time.perf_counter() - t0
    nq = q0.shape[0]
    ans, online, maint = og.SearchLoop(q0, k, STEP, PARALLEL)
    timed = ans[warmup:]
    gt = pm.knn(v, q0[warmup:], K_TOP, ctx)
    same = (timed == answers0).all(axis=1)
    out = {"value": nq / (online + maint), "unit": "queries/s", "cores": 1, "kind": "port",
           "identical_answers": {"queries": int(len(same)), "identical": int(same.sum()),
                                 "frac": round(float(same.mean()), 6)},
           "recall_at_10": round(float(compute_recall(gt, timed, K_TOP)), 4),
           "gpu_recall_at_10_same_queries": round(float(compute_recall(gt, answers0, K_TOP)), 4),
           "sample": f"session 0's workload replayed: {nq} private queries ({warmup} warm-up + {nq - warmup} timed, "
                     f"same seeds) after one {prep:.2f}s preprocessing; online {online:.2f}s + "
                     f"maintenance {maint:.2f}s"}
    return out


def cpu_baseline_all_cores(v, g, out):
    """The oracle on all the box's host cores (16 per GPU): one independent
    client per core over the same data, like the GPU's sessions."""
    from oracle import oracle as O
    nq = 46
    # all host cores (the box's CPU share: 16 per GPU): one independent oracle
    # client per core, like the GPU's sessions, over the same data; each runs
    # the same sample shape (one preprocessing, then 46 queries = two
    # maintenance windows); ctypes releases the GIL, so the C loops run in parallel
    import threading
    ncores = min(16, os.cpu_count() or 1)
    nq1 = nq
    qall = make_queries(v, ncores * nq1, seed=999)
    res = [None] * ncores

    def client(i):
        oc = O.Graph(v, g, pir_seed=1000 + i, search_seed=2000 + i)
        oc.Preprocess()
        _, on, mt = oc.SearchLoop(qall[i * nq1:(i + 1) * nq1], K_TOP, STEP, PARALLEL)
        res[i] = (on, mt)
        del oc

    th = [threading.Thread(target=client, args=(i,)) for i in range(ncores)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    wall = time.perf_counter() - t0
    on_sum = sum(r[0] for r in res)
    mt_sum = sum(r[1] for r in res)
    out["all_cores"] = {"value": round(ncores * nq1 / (on_sum + mt_sum) * ncores, 2), "cores": ncores,
                        "wall_value": round(ncores * nq1 / wall, 2),
                        "note": f"{ncores} concurrent oracle clients x {nq1} queries (two maintenance windows each); "
                                "value = queries / (mean per-client online + maintenance time) summed over "
                                "clients; wall_value includes each client's first preprocessing"}
    return out


def main():
    # The contract is ONE JSON line on rank 0's stdout; native libraries write
    # banners there (gloo prints its peer-connection lines at rendezvous), so
    # file descriptor 1 points at stderr for the whole run and the line goes
    # to the saved descriptor.
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sessions", type=int, default=SESSIONS, help="client sessions served per GPU")
    ap.add_argument("--mode", choices=["batched", "concurrent"], default="batched",
                    help="batched: lock-step groups sharing one step per round (default); "
                         "concurrent: one host thread + stream + own steps per session")
    ap.add_argument("--groups", type=int, default=GROUPS, help="lock-step groups (batched mode)")
    ap.add_argument("--threads", type=int, default=THREADS, help="host worker threads (batched mode)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config2", action="store_true", help="skip the MS-MARCO-shaped batch-PIR block")
    ap.add_argument("--no-single", action="store_true", help="skip the one-client latency block")
    ap.add_argument("--no-bigann", action="store_true", help="skip the BIGANN-100M / 1B batch-PIR blocks")
    ap.add_argument("--no-config0", action="store_true", help="skip the InnerProduct scan block")
    ap.add_argument("--big-sessions", type=int, default=0, help="cap on the BIGANN blocks' sessions per GPU")
    ap.add_argument("--bigann-blocks", default="3,4",
                    help="which BIGANN blocks run: configs[3] (100M) and/or configs[4] (1B), e.g. '3' for a "
                         "multi-rank rehearsal on one GPU, where the 1B layout's shards do not fit")
    ap.add_argument("--big-groups", type=int, default=0, help="lock-step teams of the BIGANN blocks (0: BIG_GROUPS)")
    ap.add_argument("--combine", choices=["rccl", "torch-rccl", "gloo"], default="rccl",
                    help="collective of the sharded BIGANN rounds: rccl = the library's own RCCL communicators "
                         "(pm_rccl_combine), torch-rccl = torch.distributed's nccl group through a callback, "
                         "gloo = host tensors (e.g. ranks sharing one GPU)")
    ap.add_argument("--bigann-budget-s", type=float, default=400.0,
                    help="wall-clock budget of the BIGANN blocks; past it the line is written and the run ends")
    ap.add_argument("--no-combine-probe", action="store_true",
                    help="skip the world-1 comparison of the two RCCL combine paths (BIGANN-100M block)")
    ap.add_argument("--kernel-timing-sample", action="store_true",
                    help="kernel-timing pass: events on every 7th shared step of each team only")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the kernel-timing pass (no rooflines)")
    ap.add_argument("--kernel-timing-in-value", action="store_true",
                    help="time every kernel with events inside the timed region itself (round-3 behaviour: "
                         "the events cost 5-7 %% of the rate) instead of in a separate pass")
    ap.add_argument("--no-msmarco-search", action="store_true", help="skip the MS-MARCO d=192 private-search block")
    ap.add_argument("--ms-sessions", type=int, default=0, help="MS-MARCO private-search sessions (0: MS_SESSIONS)")
    ap.add_argument("--ms-groups", type=int, default=0, help="MS-MARCO private-search lock-step teams (0: MS_GROUPS)")
    ap.add_argument("--stagger-teams", action="store_true", default=os.environ.get("PM_BENCH_STAGGER") == "1",
                    help="desynchronise the teams' maintenance windows (extra warm-up queries per team)")
    ap.add_argument("--graph", choices=["built", "random"], default="built",
                    help="GPU-built kNN+robustPrune graph (default) or the reference's synthetic random graph")
    args = ap.parse_args()
    S = max(1, args.sessions)

    dist, rank, ws, local = dist_init()
    # torch before libpacmann.so: both then share torch's HIP runtime (the same
    # SONAME; loaded the other way round, torch sees no GPU), which the
    # BIGANN blocks' RCCL combine probe needs
    import torch  # noqa: F401
    import pacmann_amd as pm

    ctx0 = pm.Context(local)
    v, g, gbuild = make_data(rank, args.graph, ctx0)
    nq = args.warmup + args.steps + KT_QUERIES + PROFILE_QUERIES
    queries = make_queries(v, S * nq + 64, seed=300 + rank)
    qsess = queries[:S * nq].reshape(S, nq, -1)
    # session 0 owns the graph and the server DB (GraphANNFrontend.Preprocess:
    # DB packing + first hint preprocessing); sessions 1..S-1 are further
    # clients over the same device DB, each with its own keys and hint state
    base = pm.PIRGraphInfo(v, g, pir_seed=11 + 97 * rank, search_seed=12 + 97 * rank, ctx=ctx0)
    base.Preprocess()
    sess = [base] + [base.Session(11 + 97 * rank + i, 12 + 97 * rank + i, pm.Context(local)) for i in range(1, S)]
    for s_ in sess[1:]:
        s_.Preprocess()
    ctxs = [s_.ctx for s_ in sess]

    def serve(qq):
        if args.mode == "batched":
            return pm.search_loop_batched(sess, qq, K_TOP, STEP, PARALLEL, args.groups, args.threads)
        return pm.search_loop_sessions(sess, qq, K_TOP, STEP, PARALLEL)
    if args.warmup:
        serve(qsess[:, :args.warmup])
    stagger = None
    if args.stagger_teams and args.mode == "batched" and args.groups > 1:
        # Desynchronise the teams' maintenance windows (a server's clients do not
        # all re-preprocess at the same query): team g serves g * step extra
        # warm-up queries, so its trigger (private-search.go:226-232, every 23
        # queries) falls `g * step` queries earlier inside the timed region, and
        # the other teams keep querying while its maintenance runs.  Every
        # session still re-preprocesses exactly once in the region (asserted in
        # maintenance_in_region).
        window = int(base.PIR.stats()["SupportBatchNum"] // (STEP * PARALLEL))
        stride = max(1, min(args.steps, window) // args.groups)
        stagger = {"teams": args.groups, "extra_warmup_queries_per_team": []}
        G = args.groups
        for g in range(1, G):
            s0, s1 = S * g // G, S * (g + 1) // G
            extra = g * stride
            xq = make_queries(v, (s1 - s0) * extra, seed=7000 + g).reshape(s1 - s0, extra, -1)
            pm.search_loop_batched(sess[s0:s1], xq, K_TOP, STEP, PARALLEL, 1, min(args.threads, s1 - s0))
            stagger["extra_warmup_queries_per_team"].append(extra)
        stagger["extra_warmup_queries_per_team"].insert(0, 0)
    progress(f"SIFT1M: {S} sessions ready, warm-up done; timed region")

    # `value` is measured with no per-launch events (timing level 0): the
    # events' dispatch-packet and completion handling cost 5-7 % of the rate
    # (profiles/r03/README.md "kernel timing").  The kernels are timed in a
    # separate pass right after it (below) over the same sessions, teams and
    # launch shapes.
    in_value = args.kernel_timing_in_value and not args.no_kernel_timing
    kt_level = 3 if args.kernel_timing_sample else 2
    prep0 = sum(s_.PIR.stats()["PrepCount"] for s_ in sess)
    for c in ctxs:
        c.timing_reset()
        c.timing(kt_level if in_value else 0)
    if dist:
        dist.barrier()
    for c in ctxs:
        c.sync()
    t0 = time.perf_counter()
    answers, _, online, maint = serve(qsess[:, args.warmup:args.warmup + args.steps])
    for c in ctxs:
        c.sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for c in ctxs:
        c.timing(False)
    prep_in_region = sum(s_.PIR.stats()["PrepCount"] for s_ in sess) - prep0

    def tsum(name, cs=ctxs):
        r = [c.timing_get(name) for c in cs]
        return tuple(sum(x[i] for x in r) for i in range(3))

    htime = {k: tsum(k) for k in HOST}
    prep_sets = tsum("host_prep_sets")
    nsteps = steps_region = htime["host_step_launch"][0]   # shared steps run in the timed region (all teams)
    ktime = {k: tsum(k) for k in KERNELS}
    kt_wall = elapsed   # the wall time the kernels were timed over
    kt_pass = None
    kt_timeline = None
    if not in_value and not args.no_kernel_timing:
        # the kernel-timing pass: KT_QUERIES more queries of every session with
        # events on every launch (one maintenance of every session inside)
        progress("SIFT1M kernel-timing pass")
        w0 = args.warmup + args.steps
        for c in ctxs:
            c.timing_reset()
            c.timing(kt_level)
        for c in ctxs:
            c.sync()
        tk = time.perf_counter()
        serve(qsess[:, w0:w0 + KT_QUERIES])
        for c in ctxs:
            c.sync()
        tk = time.perf_counter() - tk
        for c in ctxs:
            c.timing(False)
        # the pass's GPU timeline (every timed launch's start / end: the
        # answers' union time and the query phase's busy share, below;
        # PM_TIMELINE=<file> keeps it for tools/timeline.py)
        tl_path = os.environ.get("PM_TIMELINE") or os.path.join(
            tempfile.gettempdir(), f"pm_timeline_{os.getpid()}.csv")
        try:
            for c in ctxs:
                c.timing_timeline(tl_path)
            kt_timeline = read_timeline(tl_path)
        except Exception as e:   # diagnostics only
            kt_timeline = {"error": f"{type(e).__name__}: {e}"}
        if not os.environ.get("PM_TIMELINE") and os.path.exists(tl_path):
            os.remove(tl_path)
        ktime = {k: tsum(k) for k in KERNELS}
        kt_pass = {"queries_per_session": KT_QUERIES, "wall_s": round(tk, 4),
                   "private_queries_per_s": round(S * KT_QUERIES / tk, 2),
                   "steps": tsum("host_step_launch")[0], "maintenance_sets": tsum("host_prep_sets")[0]}
        nsteps = kt_pass["steps"]
        kt_wall = tk
    # --kernel-timing-sample (timing level 3; measured no faster than level 2 on
    # the SIFT1M line, 13.1-15.2K vs 15.4-15.5K q/s, so not the default): the
    # shared steps' kernels carry events on every 7th step of
    # each team (pm_ctx::timed_ext); their launch averages come from that sample,
    # their region totals (kernel_ms, the dominant kernel, the aggregate rate) are
    # the sample scaled to every step of the region
    ktot = {k: (ktime[k][1], ktime[k][2]) for k in KERNELS}   # region totals: ms, bytes
    sampled = {}
    for k in STEP_KERNELS:
        n, ms, by = ktime[k]
        if n and nsteps > n:
            sampled[k] = n
            ktot[k] = (ms * nsteps / n, by * nsteps / n)
    # the same kernels with ONE lock-step group alone on the GPU (no other
    # group's kernels beside them), and one client's maintenance alone: the
    # isolated per-launch times beside the contended ones above
    isolated = one_prf = None
    if args.mode == "batched" and not args.no_kernel_timing:
        gsz = max(1, S // max(1, args.groups))
        grp = sess[:gsz]
        for c in ctxs:
            c.timing_reset()
        grp[0].ctx.timing(2)
        w0 = args.warmup + args.steps + KT_QUERIES
        pm.search_loop_batched(grp, qsess[:gsz, w0:w0 + PROFILE_QUERIES], K_TOP, STEP, PARALLEL, 1,
                               min(args.threads, gsz))
        grp[0].ctx.timing(False)
        one = sess[-1]
        one.ctx.timing_reset()
        one.ctx.timing(1)
        one.PIR.Preprocessing()
        one.ctx.timing(False)
        isolated = {"sessions": gsz, "queries_each": PROFILE_QUERIES, "kernel_avg_us": {}}
        for k in ("hint_match", "resolve", "match_resolve", "answer", "team_round"):
            n, ms, by = grp[0].ctx.timing_get(k)
            if n:
                isolated["kernel_avg_us"][k] = round(ms / n * 1e3, 3)
                if by:
                    ach = (by / n) / (ms / n / 1e3) / 1e9
                    isolated[f"{k}_roofline"] = {"achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                                                 "alg_bytes_per_launch": by / n}
        for k in ("prep_offsets", "prep_fold", "prep_repl"):
            n, ms, _ = one.ctx.timing_get(k)
            if n:
                isolated["kernel_avg_us"][f"{k}_one_client"] = round(ms / n * 1e3, 3)
        one_prf = one.ctx.timing_get("prep_offsets")
    # recall@10 of every timed answer against exact kNN (ComputeRecall, build_graph.go:821-863)
    from pacmann_amd.report import compute_recall
    tq = qsess[:, args.warmup:args.warmup + args.steps].reshape(-1, DIM)
    gt = pm.knn(v, tq, K_TOP, ctx0)
    recall = compute_recall(gt, answers.reshape(-1, K_TOP), K_TOP)
    # the reference's own accounting, one client alone (latency view; not `value`)
    single = None
    if rank == 0 and not args.no_single:
        n1 = min(args.steps, 50)
        sq = queries[S * nq:S * nq + n1] if S * nq + n1 <= len(queries) else qsess[0, :n1]
        t1 = time.perf_counter()
        _, on1, mt1 = base.SearchLoop(sq, K_TOP, STEP, PARALLEL)
        base.ctx.sync()
        t1 = time.perf_counter() - t1
        single = {"queries_per_s": round(n1 / t1, 2), "ms_per_query": round(t1 / n1 * 1e3, 4),
                  "online_s_per_query": round(on1 / n1, 6), "maintenance_s_per_query": round(mt1 / n1, 6),
                  "queries": n1}
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_q = args.steps * S * ws
    value = total_q / elapsed
    # The driver's 20-query region holds one maintenance per session, the steady
    # state one per 23 queries (private-search.go:226-232): the same region with
    # its maintenance time scaled to that cadence, for reference (not `value`)
    at_cadence = None
    window = int(base.PIR.stats()["SupportBatchNum"] // (STEP * PARALLEL))
    per_sess = prep_in_region / S if S else 0
    if args.mode == "batched" and per_sess > 0 and window > 0 and len(maint):
        m_reg = float(np.max(maint))   # merged sets: every session's maintenance time is the sets' GPU span
        m_ss = m_reg * (args.steps / window) / per_sess
        at_cadence = {"value": round(total_q / max(elapsed - m_reg + m_ss, 1e-9), 2),
                      "region_maintenance_s": round(m_reg, 4), "maintenances_per_session": round(per_sess, 3),
                      "cadence_queries": window,
                      "note": "value with the region's maintenance time scaled from maintenances_per_session to "
                              "steps / cadence_queries per session (the steady state); reference only"}
    # dominant kernel: largest device time over the timed region
    dom = max(KERNELS, key=lambda k: ktot[k][0])

    def roof(name, note=None):
        n, ms, by = ktime[name]
        if n == 0 or ms == 0 or by == 0:
            return None
        ach = (by / n) / (ms / n / 1e3) / 1e9
        grid = None
        if name == "answer" and args.mode == "batched":   # the PMC summary by launch shape: one workgroup per sub-query
            grid = answer_grid((S // max(1, args.groups)) * PARALLEL * M)
        r = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
             "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
             "launches": n, "avg_ms": round(ms / n, 5), "alg_bytes_per_launch": by / n}
        attach_traffic(r, SYMBOLS.get(name, name), grid)
        if note:
            r["note"] = note
        return r

    stats = base.PIR.stats()
    # the fold against its compulsory bytes too: the DB once plus the parities
    hints = 0
    for p in range(stats["PartitionNum"]):
        c = base.PIR.SubConfig(p)
        hints += c["PrimaryHintNum"] + c["SetSize"] * c["MaxQueryPerChunk"]
    E = (DIM + M) // 2
    fold = roof("prep_fold")
    if fold:
        # a launch folds k clients' hints at once (batched serving re-preprocesses a group's
        # triggered clients together); they share the one DB
        c0 = base.PIR.SubConfig(0)
        fold_one = sum(((c["PrimaryHintNum"] + (c["SetSize"] - 1) * c["MaxQueryPerChunk"]) * c["SetSize"] * E * 8)
                       for c in (base.PIR.SubConfig(p) for p in range(stats["PartitionNum"])))
        k = max(1, round(fold["alg_bytes_per_launch"] / fold_one))
        comp = N * E * 8 + k * hints * E * 8
        ach_c = comp / (fold["avg_ms"] / 1e3) / 1e9
        fold["clients_per_launch"] = k
        fold["compulsory"] = {"bytes": comp, "achieved": round(ach_c, 1), "frac": round(ach_c / HBM_PEAK_GBS, 4)}
        # PMC bytes of launches of this shape (k_prep_fold_rot<512>: the k clients' hints of a
        # partition in virtual groups of 5,120; XCD tiles of 4 (partition, group) pairs x 8 of the
        # 20 column slices, dealt to the 8 XCDs in turn; 1,024 threads per workgroup;
        # pm_kernels.hip prep_fold)
        H0 = c0["PrimaryHintNum"] + c0["SetSize"] * c0["MaxQueryPerChunk"]
        npv = stats["PartitionNum"] * -(-(k * H0) // 5120)
        tiles = -(-npv // 4) * -(-(E // 4) // 8)
        attach_traffic(fold, SYMBOLS["prep_fold"], 8 * -(-tiles // 8) * 32 * 1024)
        # the fold is LDS-bound, not HBM-bound: its fold bytes (one entry read per
        # (hint, chunk) pair) are ds_read_b128 reads of the staged
        # chunks; HBM carries the staging (PMC traffic) and the parity writes
        fold["bound"], fold["peak"] = "lds", LDS_B128_PEAK_GBS
        fold["frac"] = round(fold["achieved"] / LDS_B128_PEAK_GBS, 4)
        fold["hbm"] = {"traffic_vs_compulsory": round(fold["traffic"] / comp, 3) if fold.get("traffic") else None}
        fold["note"] = ("bound lds: fold bytes (hint x chunk entry reads, SURVEY.md §8d) served from LDS by "
                        "ds_read_b128 against the ~150 TB/s aggregate (MI355X_MICROARCH.md §LDS); 'compulsory' is "
                        "the HBM side: the DB read once plus the parity writes of the clients folded in one launch")
    ss0 = base.PIR.SubConfig(0)["SetSize"]
    prf = prf_roofline(ktime["prep_offsets"], "k_prep_offsets of the kernel-timing pass's maintenance launch", ss0)
    if prf and isolated and one_prf:
        prf["isolated_one_client"] = prf_roofline(one_prf, "one client alone", ss0)
    note = None
    if dom == "step":
        note = ("k_step runs hint match, resolution and answer of a batch-PIR step in one launch; "
                "bytes are the answer's (SURVEY.md §8d: SS*E*8 + 4*SS + 8*E per real/dummy sub-query); "
                f"avg_ms is per launch with {S} sessions' steps in flight together")
    elif dom == "answer":
        note = (f"k_answer of the shared step of {S // max(1, args.groups)} lock-step sessions (set expansion, "
                "XOR gather, decode, refresh, L2); bytes per SURVEY.md §8d: SS*E*8 + 4*SS + 8*E per sub-query")
    elif dom != "prep_fold":
        note = (f"dominant kernel by device time is {dom}, which has no §8(d) byte figure; "
                f"the roofline shown is the PIR answer kernel's")
    main_roof = roof(dom, note) if dom in ("answer", "prep_fold", "step") else roof("answer", note)
    ans_k = "step" if args.mode == "concurrent" else "answer"
    if main_roof and main_roof["kernel"] == ans_k:
        # all sessions' answer bytes over the wall time they were served in (the GPU-wide PIR-scan rate)
        agg = ktot[ans_k][1] / kt_wall / 1e9
        main_roof["aggregate"] = {"achieved": round(agg, 1), "frac": round(agg / HBM_PEAK_GBS, 4),
                                  "note": "answer bytes of every step of the kernel-timing pass / its wall time"
                                          if kt_pass else "answer bytes of every step in the timed region / its "
                                          "wall time"}
    if main_roof and main_roof["kernel"] == ans_k and isinstance(kt_timeline, dict) and "answer" in kt_timeline:
        # The device loop overlaps the teams' answers (1-2 in flight most of the
        # query phase), so a launch's own duration overstates its cost: the
        # answers' union time is what they take of the GPU
        u = kt_timeline["answer"]
        if u["union_ms"] > 0:
            ach = u["launches"] * main_roof["alg_bytes_per_launch"] / (u["union_ms"] / 1e3) / 1e9
            main_roof["union"] = {
                "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                "effective_us_per_launch": round(u["union_ms"] * 1e3 / u["launches"], 2),
                "launches": u["launches"], "union_ms": u["union_ms"],
                "note": "answer bytes of the kernel-timing pass over the union of its answer launches' "
                        "[start, end] intervals (the GPU time during which any answer ran)"}
    if main_roof and not args.no_kernel_timing:
        main_roof["composite"] = composite_floor(ktime, S, kt_pass["queries_per_session"] if kt_pass else args.steps,
                                                 base.PIR, value / ws, ss_r2=base.PIR.SubConfig(0)["SetSize"])
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "queries/s", "n_gpus": ws,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": ("synthetic SIFT-like uint8-valued f32 vectors (12-D latent mixture); "
                 + ("uniform random degree-32 graph (genRandomGraph)" if args.graph == "random"
                    else "degree-32 graph built on the GPU (exact kNN candidates + robustPrune, alpha 1.2)")),
        "config": {"workload": "SIFT1M-shaped private graph search over 16-partition batch PianoPIR",
                   "n": N, "dim": DIM, "m": M, "k": K_TOP, "step": STEP, "parallel": PARALLEL,
                   "batch_size": M, "failure_prob_log2": F, "sessions_per_gpu": S, "serving": args.mode,
                   "lockstep_groups": args.groups if args.mode == "batched" else None,
                   "parallelism": f"replicas{ws}"},
        "roofline": main_roof,
        "roofline_prep": fold,
        "roofline_prf": prf,
        "single_session": single,
        "recall_at_10": round(float(recall), 4),
        "recall_queries": int(tq.shape[0]),
        "graph_build": gbuild,
        "online_s_per_query": round(float(np.mean(online)) / args.steps, 6),
        "maintenance_s_per_query": round(float(np.mean(maint)) / args.steps, 6),
        "preprocessing_s": round(stats["PreprocessingTime"], 6),
        "kernel_ms": {k: round(ktot[k][0], 3) for k in KERNELS},
        "kernel_timing": {"step_kernels_sampled": bool(sampled), "timed_launches": sampled,
                          "launches_in_pass": nsteps,
                          "note": "the shared steps' kernels carry events on every 7th step of each team "
                                  "(pm_timing_enable level 3): per-launch averages from that sample, kernel_ms "
                                  "scaled to every step (--kernel-timing-sample)"} if sampled else None,
        "kernel_avg_us": {k: round(ktime[k][1] / ktime[k][0] * 1e3, 3) if ktime[k][0] else None for k in KERNELS},
        "host_ms": {k: round(htime[k][1], 3) for k in HOST},
        "steps_in_region": steps_region,
        # the region's maintenance: every session re-preprocesses once per 23-query window
        # (private-search.go:226-232), so `value` carries ~steps/23 maintenances per session
        "maintenance_in_region": {"preprocessings": prep_in_region, "per_session": round(prep_in_region / S, 3),
                                  "launch_sets": prep_sets[0], "clients_per_set": round(prep_sets[1] / prep_sets[0], 1)
                                  if prep_sets[0] else None,
                                  "window_queries": int(stats["SupportBatchNum"] // (STEP * PARALLEL)),
                                  "note": "fewer than one per session: the line's maintenance share is below the "
                                          "steady state's (steps shorter than a window)"
                                          if prep_in_region < S else "at least one per session"},
        "value_at_maintenance_cadence": at_cadence,
        "kernel_timing_pass": kt_pass,
        "kernel_timing_timeline": ({k: v for k, v in kt_timeline.items()
                                    if k in ("answer", "match_resolve", "team_round", "query_phase", "error")}
                                   if isinstance(kt_timeline, dict) else None),
        "maintenance_stagger": stagger,
        # result rows the host read at token time vs those whose bytes did not yet
        # match their header hash then; results are taken only after the step's
        # completion event (system-scope release), where a mismatch is an error
        # (result publication)
        "rows_check": {"seen": int(htime["host_rows_seen"][0]), "torn_at_token": int(htime["host_rows_torn"][0]),
                       "completion_waits": int(htime["host_wait_done"][0]),
                       "completion_wait_ms": round(htime["host_wait_done"][1], 3),
                       "ordered": os.environ.get("PM_PUBLISH_WAIT", "1") != "0"},
        "dominant_kernel": dom,
    }
    if isolated:
        out["isolated"] = isolated
    if not args.no_cpu_baseline and ws == 1:
        progress("SIFT1M cpu_baseline")
        cb = cpu_baseline(v, g, qsess[0, :args.warmup + args.steps], args.warmup, answers[0], ctx0,
                          11 + 97 * rank, 12 + 97 * rank)
        cpu_baseline_all_cores(v, g, cb)
        out["cpu_baseline"] = cb
    # the SIFT1M serving state is done with: free its device memory (HBM) for the other blocks
    import gc
    del sess, base, ctxs, ktime
    gc.collect()
    if ws == 1 and not args.no_config2:
        c2 = pm.Context(local)
        progress("config2 batch PIR")
        out["config2_batch_pir"] = batch_pir_msmarco(c2, not args.no_cpu_baseline)
        del c2
        gc.collect()
    if ws == 1 and not args.no_msmarco_search:
        try:
            progress("config2 MS-MARCO private search")
            out["config2_private_search"] = private_search_msmarco(local, args, not args.no_cpu_baseline)
        except Exception as e:   # recorded, never fatal to the headline line
            out["config2_private_search"] = {"error": f"{type(e).__name__}: {e}"}
        gc.collect()
    if ws == 1 and not args.no_config0:
        c0 = pm.Context(local)
        progress("config0 inner product")
        out["config0_inner_product"] = inner_product_scan(c0, not args.no_cpu_baseline)
        del c0
        gc.collect()
    # BASELINE.json configs[3] (BIGANN-100M, sharded over the ranks) and
    # configs[4] (BIGANN-1B in 8 shards), and with several ranks configs[0]
    # sharded by rows: every rank takes part
    ip_multi = ws > 1 and not args.no_config0
    if not args.no_bigann or ip_multi:
        # The headline and the single-GPU blocks are complete: their line goes to
        # stderr now, and a watchdog writes the full line (the BIGANN blocks
        # marked unfinished) and ends the process if the blocks below overrun
        # their budget, so a hang in a collective cannot lose the line.
        if rank == 0:
            progress("PARTIAL_LINE " + json.dumps(out))
        want = set() if args.no_bigann else {b.strip() for b in args.bigann_blocks.split(",")}
        wd = start_watchdog(out, rank, line_fd, args.bigann_budget_s,
                            keys=(["config0_inner_product"] if ip_multi else []) +
                                 [k for k in ("config3_bigann_100m", "config4_bigann_1b") if k[6] in want])
        pm.set_option("rccl_timeout_s", 60)   # a peer that never joins costs 60 s, not the run
        prefer = {"rccl": "native", "torch-rccl": "torch-rccl", "gloo": "gloo"}[args.combine]
        memo = {}

        def nccl_group_fn():   # the torch RCCL group, probed and agreed once (rccl_group)
            if "g" not in memo:
                memo["g"] = rccl_group(dist, local, out)
            return memo["g"]
        if ip_multi:
            try:
                progress("config0 inner product, sharded by rows")
                c0 = pm.Context(local)
                wd.put("config0_inner_product", inner_product_scan_sharded(c0, dist, rank, ws, local, nccl_group_fn))
                del c0
                gc.collect()
            except Exception as e:   # recorded, never fatal to the headline line
                wd.put("config0_inner_product", {"error": f"{type(e).__name__}: {e}"})
        for key, nm, n_entries in (("config3_bigann_100m", "BIGANN-100M-shaped (configs[3])", 100_000_000),
                                   ("config4_bigann_1b", "BIGANN-1B-shaped (configs[4])", 1_000_000_000)):
            if key[6] not in want:
                continue
            try:
                progress(key)
                lay = bigann_layout(key, ws, rank)
                rgroup = replica_groups(dist, ws, lay["layout"]) if dist and lay["replicas"] > 1 else None
                wd.put(key, bigann_search(key, nm, n_entries, lay, rank, ws, local, dist, prefer, args,
                                          nccl_group_fn=nccl_group_fn if dist else None,
                                          replica_group=None if rgroup is None else rgroup[lay["replica"]]))
            except Exception as e:   # recorded, never fatal to the headline line
                wd.put(key, {"error": f"{type(e).__name__}: {e}"})
        if not wd.fire():   # the watchdog already wrote the line and is ending the process
            return
    if rank == 0:
        sys.stdout.flush()
        os.write(line_fd, (json.dumps(out) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
