"""Report / recall / answer-file parity (private-search.go:
286-331, graphann/build_graph.go:821-863, graphann/loader.go:217-364).

The fixture tests/golden/private_search_report_sift1m.txt is the first block
of the reference's private-search-report.txt (its SIFT1M run).  That file
predates the "** Random Seed" line private-search.go:312 prints today, so the
comparison drops that one line.  Parameter-derived fields come from the
oracle's accounting (dummy preprocessing, no DB scan); the measured fields
(preparation time, computation time, recall) are the report's own values."""
import os

import numpy as np

from pacmann_amd.report import (compute_recall, format_report, load_int_matrix, report_fields,
                                save_int_matrix)

GOLD = os.path.join(os.path.dirname(__file__), "golden", "private_search_report_sift1m.txt")


def test_report_block_matches_reference(oracle):
    N, E = 1_000_000, 80
    b = oracle.SimpleBatchPianoPIR(N, E * 8, 32, np.zeros(N * E, np.uint64), 8)
    b.DummyPreprocessing()
    s = b.stats()
    s.update({"DBSize": N, "DBEntryByteNum": E * 8, "PreprocessingTime": 2.639725})
    f = report_fields(s, n=N, k=10, step=20, parallel=3)
    assert f["window"] == 23
    got = format_report(rtt_ms=50, seed=1, avg_time=0.055917, recall=0.939501, **f)
    got = [ln for ln in got.splitlines() if not ln.startswith("** Random Seed")]
    want = open(GOLD).read().splitlines()
    assert got == want


def test_compute_recall_skips_repeats():
    gnd = [[1, 2, 3, 4], [5, 6, 7, 8]]
    resp = [[1, 1, 2, 9], [8, 7, 6, 5]]
    # row 0: 1 hit, repeat skipped, 2 hit, 9 miss -> 2/4; row 1: 4/4
    assert compute_recall(gnd, resp, 4) == float(np.float32((np.float32(0.5) + np.float32(1.0)) / 2))
    assert compute_recall([[0, 1, 2]], [[3, 4, 5]], 3) == 0.0


def test_int_matrix_files_round_trip(tmp_path):
    m = np.arange(12, dtype=np.int64).reshape(3, 4) * 7 - 5
    for ext in (".npy", ".txt"):
        p = str(tmp_path / f"a{ext}")
        save_int_matrix(p, m)
        assert np.array_equal(load_int_matrix(p, 3, 4), m)
    txt = open(str(tmp_path / "a.txt")).read().splitlines()
    assert txt[0] == "-5 2 9 16 "   # SaveGraphToTxtFile: "%d " per field, newline per row
    iv = tmp_path / "g.ivecs"
    rows = np.array([[3, 1, 2, 3], [3, 4, 5, 6]], dtype=np.uint32)   # dim-prefixed uint32 rows
    rows.tofile(str(iv))
    assert np.array_equal(load_int_matrix(str(iv), 2, 3), [[1, 2, 3], [4, 5, 6]])


def test_mrr_at_k(tmp_path):
    """reproduction/msmarco/evaluate.py semantics: first relevant docid per
    query (qrels setdefault), first hit rank, invalid ids never match, text
    and .npy result files, the docid listing."""
    import numpy as np
    from pacmann_amd.report import mrr_at_k, read_qrels, read_queries_tsv, read_results
    (tmp_path / "q.tsv").write_text("10\twhat is a\n11\tb c\n12\tnone\n")
    (tmp_path / "qrels").write_text("10 0 D7 1\n10 0 D9 1\n11 0 D1 1\n12 0 D5 1\n")
    docids = np.array([f"D{i}" for i in range(10)])
    res = np.array([[3, 9, 7], [1, -4, 2], [12, 0, 0]])
    np.save(tmp_path / "r.npy", res)
    (tmp_path / "r.txt").write_text("\n".join(" ".join(map(str, r)) for r in res) + "\n")
    qs, qr = read_queries_tsv(tmp_path / "q.tsv"), read_qrels(tmp_path / "qrels")
    assert qr["10"] == "D7"
    for f in ("r.npy", "r.txt"):
        r = read_results(str(tmp_path / f), 3, 3)
        out = mrr_at_k(r, qs, qr, docids, output_docids=str(tmp_path / "ids.txt"))
        assert out["ranked_queries"] == 2 and abs(out["mrr"] - (1 / 3 + 1) / 3) < 1e-12
    listing = (tmp_path / "ids.txt").read_text().splitlines()
    assert listing[0] == "Query: 10 what is a" and "INVALID_VECTOR_ID" in listing
    import pytest
    with pytest.raises(ValueError):
        read_results(str(tmp_path / "r.npy"), 3, 4)
