"""The GetGraphInfo plugin surface (graphann/search.go:20-25) of PIRGraphInfo
(private-search.go:336-531) through its C entry points: pm_graph_get_metadata,
pm_graph_get_vertex_info (GetVertexInfo, :441-506: batch-PIR fetch + the
Entry2VectorAndNeighbors decode, :418-439, plus the L2 distance to a query in
the reference's order) and pm_graph_get_start_vertex (GetStartVertex,
:508-531), against the oracle's restatement of the same methods."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, DIM, M = 20_000, 128, 32


def _data(seed):
    from pacmann_amd.synth import random_graph, sift_like_vectors
    return sift_like_vectors(N, DIM, seed=seed), random_graph(N, M, seed=seed + 1)


def test_get_vertex_info_vs_oracle(ctx, oracle):
    """60 GetVertexInfo batches of 96 ids (the search's batch shape, with
    repeats inside a batch and across batches) — past the batch layer's
    re-preprocessing trigger — give the oracle's vectors and neighbour lists
    bit for bit, zeros exactly where the fetch failed, GPU distances equal to
    the oracle's L2Dist of the decoded vectors, and the same counters."""
    import pacmann_amd as pm
    v, g = _data(61)
    gi = pm.PIRGraphInfo(v, g, pir_seed=71, search_seed=72, ctx=ctx)
    og = oracle.Graph(v, g, pir_seed=71, search_seed=72)
    gi.Preprocess()
    og.Preprocess()
    assert gi.GetMetadata() == og.GetMetadata() == (N, DIM, M)
    ids_g, vec_g, nb_g = gi.GetStartVertex()
    ids_o, vec_o, nb_o = og.GetStartVertex()
    assert len(ids_g) == int(np.sqrt(N))
    assert np.array_equal(ids_g, ids_o) and np.array_equal(vec_g, vec_o) and np.array_equal(nb_g, nb_o)
    assert np.array_equal(vec_g, v[ids_g]) and np.array_equal(nb_g, g[ids_g])
    rng = np.random.default_rng(73)
    nok = 0
    for b in range(60):
        ids = rng.integers(0, N, size=96)
        ids[5] = ids[1]
        if b:
            ids[10:14] = prev[20:24]   # noqa: F821  (repeats across batches: the local cache)
        q = v[rng.integers(0, N)] + rng.normal(0, 8, DIM).astype(np.float32)
        vg, ng, ok, d = gi.GetVertexInfo(ids, q)
        vo, no = og.GetVertexInfo(ids)
        assert np.array_equal(vg.view(np.uint32), vo.view(np.uint32)), b
        assert np.array_equal(ng, no), b
        good = (no == g[ids]).all(axis=1)
        assert np.array_equal(ok, good), b   # success flag <=> the true row (the reference's check)
        assert not vg[~ok].any() and not ng[~ok].any(), b
        want = np.array([oracle.l2dist(vo[i], q) if ok[i] else 0.0 for i in range(96)], dtype=np.float32)
        assert np.array_equal(d.view(np.uint32), want.view(np.uint32)), b
        nok += int(ok.sum())
        prev = ids
    assert nok > 0.75 * 60 * 96   # the rest: overflow drops (6 sub-queries per partition per batch)
    assert gi.counts() == og.counts()
    sg, so = gi.PIR.stats(), og.pir().stats()
    for k in ("FinishedBatchNum", "QueriesMadeInPartition", "PrepCount"):
        assert sg[k] == so[k], k
    assert sg["PrepCount"] >= 2


def test_get_vertex_info_nonprivate(ctx, oracle):
    """Non-private mode (private-search.go:445-455): the rows come straight
    from the graph, every id succeeds, distances in the reference's L2 order."""
    import pacmann_amd as pm
    v, g = _data(81)
    gi = pm.PIRGraphInfo(v, g, nonprivate=True, pir_seed=5, search_seed=6, ctx=ctx)
    gi.Preprocess()
    ids = np.random.default_rng(3).integers(0, N, size=200)
    q = v[7] + 1
    vg, ng, ok, d = gi.GetVertexInfo(ids, q)
    assert ok.all() and np.array_equal(vg, v[ids]) and np.array_equal(ng, g[ids])
    want = oracle.l2_batch(q, v[ids])
    assert np.array_equal(d.view(np.uint32), want.view(np.uint32))
    vg2, ng2, ok2 = gi.GetVertexInfo(ids[:10])
    assert np.array_equal(vg2, v[ids[:10]]) and ok2.all()


def test_get_vertex_info_rejects(ctx):
    import pacmann_amd as pm
    v, g = _data(91)
    gi = pm.PIRGraphInfo(v, g, pir_seed=5, search_seed=6, ctx=ctx)
    with pytest.raises(RuntimeError, match="not preprocessed"):
        gi.GetVertexInfo([1, 2, 3])
    gi.Preprocess()
    with pytest.raises(RuntimeError, match="out of range"):
        gi.GetVertexInfo([N])
