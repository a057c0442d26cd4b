"""pacmann_amd.loader against the edge behaviour of graphann/loader.go (CPU)."""
import numpy as np
import pytest

from pacmann_amd import loader as L


def vecs_bytes(rows, dtype):
    out = bytearray()
    for r in rows:
        r = np.asarray(r, dtype=dtype)
        out += np.int32(r.size).tobytes() + r.tobytes()
    return bytes(out)


def test_bvecs_uniform_and_short(tmp_path):
    rng = np.random.default_rng(0)
    v = rng.integers(0, 256, size=(50, 16), dtype=np.uint8)
    p = tmp_path / "a.bvecs"
    p.write_bytes(vecs_bytes(v, np.uint8))
    got = L.load_float32_matrix(p, 50, 16)
    assert got.dtype == np.float32 and np.array_equal(got, v.astype(np.float32))
    # asking for more rows than stored: the rest stay zero (LoadBvecsFile :40-44)
    got = L.load_bvecs(p, 60, 16)
    assert np.array_equal(got[:50], v.astype(np.float32)) and not got[50:].any()
    # a record longer than dim is cut (copy), shorter leaves zeros
    p2 = tmp_path / "b.bvecs"
    p2.write_bytes(vecs_bytes([np.arange(20), np.arange(5)], np.uint8))
    got = L.load_bvecs(p2, 2, 8)
    assert np.array_equal(got[0], np.arange(8, dtype=np.float32))
    assert np.array_equal(got[1], np.r_[np.arange(5), np.zeros(3)].astype(np.float32))


def test_fvecs_and_ivecs(tmp_path):
    rng = np.random.default_rng(1)
    v = rng.standard_normal((30, 12)).astype(np.float32)
    p = tmp_path / "a.fvecs"
    p.write_bytes(vecs_bytes(v, np.float32))
    assert np.array_equal(L.load_float32_matrix(p, 30, 12), v)
    assert L.load_fvecs(p, 40, 12).shape == (30, 12)   # stops at EOF: fewer rows
    ids = rng.integers(0, 2**31, size=(10, 100), dtype=np.uint32)
    q = tmp_path / "gt.ivecs"
    q.write_bytes(vecs_bytes(ids, np.uint32))
    assert np.array_equal(L.load_int_matrix(q, 10, 100), ids.astype(np.int64))
    with pytest.raises(L.LoaderError):
        L.load_ivecs(q, 11, 100)   # the Go reader panics on a short ivecs file


def test_txt(tmp_path):
    p = tmp_path / "v.txt"
    p.write_text("1.5 2 3\n0.1 -4e2 5\n")
    got = L.load_float32_matrix(p, 3, 3)
    assert got.dtype == np.float32
    assert np.array_equal(got[:2], np.array([[1.5, 2, 3], [0.1, -400, 5]], dtype=np.float32))
    assert not got[2].any()   # missing lines stay zero
    bad = tmp_path / "bad.txt"
    bad.write_text("1 2\n")
    with pytest.raises(L.LoaderError):
        L.load_txt_float32(bad, 1, 3)
    g = tmp_path / "g.txt"
    g.write_text("1 2 3\n4 5 6\n")
    assert np.array_equal(L.load_graph(g, 2, 3), [[1, 2, 3], [4, 5, 6]])


def test_npy(tmp_path):
    rng = np.random.default_rng(2)
    v = rng.standard_normal((20, 8))
    p = tmp_path / "v.npy"
    np.save(p, v)
    got = L.load_float32_matrix(p, 15, 8)
    assert np.array_equal(got, v[:15].astype(np.float32))
    with pytest.raises(L.LoaderError):
        L.load_npy_float32(p, 21, 8)   # fewer rows than asked
    p32 = tmp_path / "v32.npy"
    np.save(p32, v.astype(np.float32))
    with pytest.raises(L.LoaderError):
        L.load_npy_float32(p32, 5, 8)  # gonpy GetFloat64 needs float64
    with pytest.raises(L.LoaderError):
        L.load_float32_matrix(tmp_path / "v.bin", 1, 1)


def test_graph_writers_round_trip(tmp_path):
    rng = np.random.default_rng(3)
    g = rng.integers(0, 10**6, size=(7, 5))
    L.save_graph(tmp_path / "g.npy", g)
    a = np.load(tmp_path / "g.npy", allow_pickle=False)
    assert a.dtype == np.int32 and np.array_equal(a, g)
    assert np.array_equal(L.load_graph(tmp_path / "g.npy", 7, 5), g)
    L.save_graph(tmp_path / "g.txt", g)
    text = (tmp_path / "g.txt").read_text()
    assert text.splitlines()[0] == "".join(f"{x} " for x in g[0])   # "%d " per entry (:339)
    assert np.array_equal(L.load_graph(tmp_path / "g.txt", 7, 5), g)
    np.save(tmp_path / "g64.npy", g.astype(np.int64))
    with pytest.raises(L.LoaderError):
        L.load_graph(tmp_path / "g64.npy", 7, 5)   # GetInt32 needs int32


def test_vecs_reads_only_the_first_records(tmp_path, monkeypatch):
    """A base file much larger than n (bigann_base.bvecs is 132 GB; the SIFT1M
    run reads its first 1e6 records): the reader maps the file and touches
    only the first n records, so a ragged or garbled record after them does
    not matter, and no whole-file array is allocated."""
    rng = np.random.default_rng(7)
    head = rng.integers(0, 256, size=(20, 16), dtype=np.uint8)
    tail = rng.integers(0, 256, size=(5000, 16), dtype=np.uint8)
    p = tmp_path / "big.bvecs"
    p.write_bytes(vecs_bytes(head, np.uint8) + vecs_bytes(tail, np.uint8) + b"\x07\x00\x00\x00garbage")
    calls = []
    real = np.fromfile
    monkeypatch.setattr(np, "fromfile", lambda *a, **k: calls.append(a) or real(*a, **k))
    got = L.load_bvecs(p, 20, 16)
    assert np.array_equal(got, head.astype(np.float32)) and not calls
    f = tmp_path / "big.fvecs"
    fv = rng.standard_normal((3000, 8)).astype(np.float32)
    f.write_bytes(vecs_bytes(fv, np.float32) + vecs_bytes([np.arange(3)], np.float32))
    assert np.array_equal(L.load_fvecs(f, 10, 8), fv[:10])   # the ragged last record is never read
    i = tmp_path / "big.ivecs"
    iv = rng.integers(0, 2**31, size=(100, 4), dtype=np.uint32)
    i.write_bytes(vecs_bytes(iv, np.uint32) + b"\x01\x02")
    assert np.array_equal(L.load_ivecs(i, 7, 4), iv[:7].astype(np.int64))
