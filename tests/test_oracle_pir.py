"""The oracle passes the reference's own PIR tests (pianopir/pir_test.go),
restated at the same sizes, and its committed transcripts."""
import hashlib

import numpy as np

from tests.golden_io import load_golden


def test_pir_basic(oracle):
    """TestPIRBasic (pir_test.go:9-58): DB 18,750 x 4 words, F=40, MaxQueryNum
    random queries, every answer == rawDB[idx]."""
    N, E = 18750, 4
    db = np.random.default_rng(0).integers(0, 2**64, size=N * E, dtype=np.uint64)
    p = oracle.PianoPIR(N, E * 8, db, 40, seed=3)
    cfg = p.Config()
    assert (cfg["ChunkSize"], cfg["SetSize"], cfg["MaxQueryNum"]) == (512, 40, 1347)
    p.Preprocessing()
    rng = np.random.default_rng(1)
    for _ in range(cfg["MaxQueryNum"]):
        idx = int(rng.integers(0, N))
        out, st = p.Query(idx, True)
        assert st == 0
        assert np.array_equal(out, db[idx * E:(idx + 1) * E])


def test_batch_pir_basic(oracle):
    """TestBatchPIRBasic (pir_test.go:60-202): 1M x 16 words, fill i, F=20."""
    N, E, B = 1_000_000, 16, 32
    db = np.repeat(np.arange(N, dtype=np.uint64), E)
    p = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, 20, seed=5)
    p.Preprocessing()
    s = p.stats()
    P, PS = s["PartitionNum"], s["PartitionSize"]
    assert (P, PS) == (16, 62500)
    rng = np.random.default_rng(2)
    view = db.reshape(N, E)
    q = np.array([i * PS + rng.integers(0, PS) for i in range(P)], np.uint64)
    out, _ = p.Query(q)
    assert np.array_equal(out, view[q])
    q = np.array([i * PS + rng.integers(0, PS) for i in range(P) for _ in range(4)], np.uint64)
    out, _ = p.Query(q)
    assert np.array_equal(out, view[q])
    q = rng.choice(PS, size=B, replace=False).astype(np.uint64)
    out, _ = p.Query(q)
    assert np.array_equal(out[:2], view[q[:2]])
    assert not out[2:].any()


def test_batch_pir_dropped_and_padded(oracle):
    """queryNumToMake = len/PartitionNum (batch-pir.go:175): a batch shorter
    than PartitionNum makes no queries at all; dummies pad short partitions."""
    N, E = 20000, 4
    db = np.random.default_rng(3).integers(0, 2**64, size=N * E, dtype=np.uint64)
    p = oracle.SimpleBatchPianoPIR(N, E * 8, 32, db, 8, seed=1)
    p.Preprocessing()
    out, _ = p.Query(np.arange(10, dtype=np.uint64))
    assert not out.any()
    assert p.stats()["QueriesMadeInPartition"] == 0


def test_pir_transcript_golden(oracle):
    g = load_golden("pir_transcript")
    N, E = int(g["N"]), int(g["E"])
    db = np.random.default_rng(int(g["db_seed"])).integers(0, 2**64, size=N * E, dtype=np.uint64)
    p = oracle.PianoPIR(N, E * 8, db, int(g["F"]), seed=int(g["seed"]))
    p.Preprocessing()
    for i, idx in enumerate(g["ids"]):
        out, st = p.Query(int(idx), True)
        assert st == g["status"][i]
        assert np.array_equal(out, g["responses"][i])
    st = p.export_state()
    dig = hashlib.sha256(b"".join(st[k].tobytes() for k in sorted(st))).hexdigest()
    assert dig == str(g["state_sha256"])


def test_batch_transcript_golden(oracle):
    g = load_golden("batch_transcript")
    N, E, B = int(g["N"]), int(g["E"]), int(g["B"])
    db = np.random.default_rng(int(g["db_seed"])).integers(0, 2**64, size=N * E, dtype=np.uint64)
    p = oracle.SimpleBatchPianoPIR(N, E * 8, B, db, int(g["F"]), seed=int(g["seed"]))
    p.Preprocessing()
    for i, q in enumerate(g["batches"]):
        out, _ = p.Query(q)
        assert np.array_equal(out, g["responses"][i])
