"""The device-generated DB spec (pm_batchpir_create_synth, include/pacmann.h):
pacmann_amd.synth_rows against a pure-Python restatement of splitmix64."""
import numpy as np

M64 = (1 << 64) - 1


def sm64(x: int) -> int:
    z = (x + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def test_synth_rows_spec():
    from pacmann_amd import synth_rows
    seed, E = 41, 80
    ids = [0, 1, 12_345_678, 10**9 - 1]
    got = synth_rows(seed, ids, E)
    k = sm64(seed + 9)
    for i, r in enumerate(ids):
        want = [sm64(k ^ (r * E + w)) for w in range(E)]
        assert got[i].tolist() == want
    assert got.dtype == np.uint64 and got.shape == (4, E)


def test_synthetic_graph_rows():
    """pm_graph_synth_rows (host code, no device) follows the synthetic graph
    spec (pm_internal.h graph_synth_elem, the reference's -input synthetic
    mode): vectors in [0, 1) with 24 random bits, neighbours in range and
    never the vertex itself, rows a pure function of (seed, vertex)."""
    import numpy as np
    import pacmann_amd as pm
    v, nb = pm.graph_synth_rows(1000, 16, 8, 5, np.arange(1000))
    assert v.dtype == np.float32 and (v >= 0).all() and (v < 1).all()
    assert np.array_equal(v * np.float32(2 ** 24), np.rint(v * np.float32(2 ** 24)))
    assert (nb < 1000).all() and not (nb == np.arange(1000)[:, None]).any()
    v2, nb2 = pm.graph_synth_rows(1000, 16, 8, 5, [999, 3])
    assert np.array_equal(v2, v[[999, 3]]) and np.array_equal(nb2, nb[[999, 3]])
    v3, _ = pm.graph_synth_rows(1000, 16, 8, 6, [3])
    assert not np.array_equal(v3, v[[3]])


def test_synthetic_graph_neighbour_spec_redraws_self_loops():
    """The neighbour rule exactly (pm_internal.h graph_synth_nb): draw
    sm64(kg ^ (v*m + k) ^ (a << 56)) % n for a = 0, 1, ... until it is not v —
    the redraw of genRandomGraph (private-search.go:54-69), uniform over the
    other n - 1 vertices.  n = 3 forces many redraws."""
    import pacmann_amd as pm
    n, dim, m, seed = 3, 4, 8, 9
    _, nb = pm.graph_synth_rows(n, dim, m, seed, np.arange(n))
    kg = sm64(seed + 11)
    redraws = 0
    for v in range(n):
        for k in range(m):
            c, a = v * m + k, 0
            x = sm64(kg ^ c) % n
            while x == v:
                a += 1
                redraws += 1
                x = sm64(kg ^ c ^ (a << 56)) % n
            assert nb[v, k] == x, (v, k)
    assert redraws > 0
