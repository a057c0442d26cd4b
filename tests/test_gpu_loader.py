"""The on-disk path into the GPU search: files written in
the reference's formats are read by `pacmann_amd.loader` exactly as
`private-search.go:main` reads them (`:107-180`: LoadFloat32Matrix for the
base and query vectors, LoadIntMatrixFromFile for the graph, the graph built
and saved when its file is missing; `:265-270`: the ground truth), then served
by the HIP path (`PIRGraphInfo` → SearchLoop) and compared with the oracle run
on the same loaded arrays.

The reference ships no vector files (SIFT1M is downloaded by SIFT-download.sh),
so the files are generated here: SIFT-like uint8 base vectors in a .bvecs file
holding more records than n (the loader reads only the first n, like the
reference's -n 1000000 over the 1B-vector base file), .fvecs queries, an .ivecs
ground truth (exact kNN on the GPU), and the graph as .npy and .txt.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _write_vecs(path, rows, dtype):
    rows = np.asarray(rows)
    n, d = rows.shape
    rec = np.zeros((n, 4 + d * np.dtype(dtype).itemsize), dtype=np.uint8)
    rec[:, :4] = np.frombuffer(np.int32(d).tobytes(), dtype=np.uint8)
    rec[:, 4:] = np.ascontiguousarray(rows, dtype=dtype).view(np.uint8).reshape(n, -1)
    rec.tofile(path)


@pytest.mark.parametrize("graph_ext", [".npy", ".txt"])
def test_files_to_gpu_search(ctx, oracle, tmp_path, graph_ext):
    import pacmann_amd as pm
    from pacmann_amd import loader, report
    from pacmann_amd.synth import sift_like_vectors

    n, extra, d, m, k, nq = 20_000, 5_000, 128, 32, 10, 30
    allv = sift_like_vectors(n + extra, d, seed=41)
    base_f = tmp_path / "base.bvecs"
    _write_vecs(base_f, allv.astype(np.uint8), np.uint8)
    rng = np.random.default_rng(42)
    qv = np.clip(np.rint(allv[rng.integers(0, n, nq)] + rng.normal(0, 6, (nq, d))), 0, 255).astype(np.float32)
    query_f = tmp_path / "query.fvecs"
    _write_vecs(query_f, qv, np.float32)

    # step 1 / 3: vectors and queries through LoadFloat32Matrix's dispatch
    vectors = loader.load_float32_matrix(str(base_f), n, d)
    queries = loader.load_float32_matrix(str(query_f), nq, d)
    assert vectors.shape == (n, d) and vectors.dtype == np.float32
    assert np.array_equal(vectors, allv[:n].astype(np.uint8).astype(np.float32))
    assert np.array_equal(queries, qv)

    # step 2: the graph file is missing -> build it (GPU), save it, read it back
    graph_f = tmp_path / f"base_{n}_{d}_{m}_graph{graph_ext}"
    assert not graph_f.exists()
    built, _ = pm.build_graph(vectors, m, ctx=ctx)
    loader.save_graph(str(graph_f), built)
    graph = loader.load_graph(str(graph_f), n, m)
    assert graph.shape == (n, m) and np.array_equal(graph, np.asarray(built, dtype=np.int64))

    # ground truth as an .ivecs file (exact kNN), read as LoadIntMatrixFromFile does
    gnd = pm.knn(vectors, queries, k, ctx=ctx)
    gnd_f = tmp_path / "gnd.ivecs"
    _write_vecs(gnd_f, np.asarray(gnd, dtype=np.int32), np.int32)
    gnd_read = loader.load_graph(str(gnd_f), nq, k)
    assert np.array_equal(gnd_read, np.asarray(gnd, dtype=np.int64))

    # step 4-6: the private search on the GPU path, answers file, recall
    g = pm.PIRGraphInfo(vectors, graph, pir_seed=7, search_seed=8, ctx=ctx)
    g.Preprocess()
    out_f = tmp_path / "answers.txt"
    res = report.private_search(g, queries, k=k, step=20, parallel=3, gnd=gnd_read, output_file=str(out_f))
    ans = res["answers"]
    assert np.array_equal(report.load_int_matrix(str(out_f), nq, k), ans)

    o = oracle.Graph(vectors, graph, pir_seed=7, search_seed=8)
    o.Preprocess()
    oa, _, _ = o.SearchLoop(queries, k, 20, 3)
    assert np.array_equal(ans, oa)
    assert g.counts() == o.counts()
    assert res["recall"] == report.compute_recall(gnd_read, oa, k)
    assert res["recall"] > 0.9, res["recall"]
