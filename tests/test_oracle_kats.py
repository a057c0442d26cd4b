"""Pin the CPU oracle against the reference's own known answers.

The reference (Go + Go asm) cannot be built here or on the GPU box (no Go
toolchain), so the oracle is pinned by:
  * FIPS-197 App. C.1 AES-128 and OpenSSL's AES (independent implementations),
  * TestXORPerf's KAT (pir_test.go:277-332) incl. xorSlices' len(src) rule,
  * TestInnerProduct (graphann_test.go:221-284): 128-element KAT + closed form,
  * the parameter / accounting figures of private-search-report.txt and
    reproduction/msmarco/README.md,
  * an independent numpy restatement of L2DistanceSIMD's order.
"""
import ctypes as C
import json
import struct

import numpy as np
import pytest

from tests.golden_io import load_golden


def test_fips197_aes128(oracle):
    rk = oracle.expand_key(bytes(range(16)))
    ct = oracle.aes128_encrypt(rk, bytes.fromhex("00112233445566778899aabbccddeeff"))
    assert ct.hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_fips197_key_schedule_last_round(oracle):
    # FIPS-197 App. A.1: key 2b7e1516..., w[40..43] = d014f9a8 c9ee2589 e13f0cc8 b6630ca6
    rk = oracle.expand_key(bytes.fromhex("2b7e151628aed2a6abf7158809cf4f3c"))
    assert rk[40:44].astype("<u4").tobytes().hex() == "d014f9a8c9ee2589e13f0cc8b6630ca6"


def test_prf_against_openssl(oracle):
    crypto = C.CDLL("libcrypto.so.3")
    rng = np.random.default_rng(0)
    for _ in range(20):
        key = rng.bytes(16)
        ak = C.create_string_buffer(244)
        assert crypto.AES_set_encrypt_key(key, 128, ak) == 0
        rk = oracle.expand_key(key)
        for _ in range(20):
            tag, x = int(rng.integers(0, 2**29)), int(rng.integers(0, 2**35))
            blk = struct.pack("<Q", (tag << 35) + x) + bytes(8)
            out = C.create_string_buffer(16)
            crypto.AES_encrypt(blk, out, ak)
            want = struct.unpack("<Q", bytes(a ^ b for a, b in zip(out.raw[:8], blk[:8])))[0]
            assert oracle.prf(rk, tag, x) == want


def test_prf_golden_vectors(oracle):
    g = load_golden("prf_vectors")
    assert len(g["vectors"]) >= 100
    for v in g["vectors"]:
        rk = oracle.expand_key(bytes.fromhex(v["key"]))
        assert oracle.prf(rk, v["tag"], v["x"]) == int(v["prf"], 16)
    # SURVEY §8c golden: key 000102..0f, tag 5, x 7
    assert oracle.prf(oracle.expand_key(bytes(range(16))), 5, 7) == 0x821E9920390BACED


def test_xor_slices_kat(oracle):
    # TestXORPerf (pir_test.go:279-290)
    p = np.full(8, 12312312, np.uint64)
    q = np.full(8, 12312, np.uint64)
    oracle.xor_slices(p, q)
    assert (p == (12312312 ^ 12312)).all()
    # count comes from len(src) floored to 4 words (aes_amd64.s:136-139)
    p = np.full(7, 12312312, np.uint64)
    q = np.full(7, 12312, np.uint64)
    oracle.xor_slices(p, q)
    assert (p[:4] == (12312312 ^ 12312)).all() and (p[4:] == 12312312).all()


def test_inner_product_kat(oracle):
    # graphann_test.go:225-247
    rng = np.random.default_rng(1)
    a = rng.integers(0, 2**32, 128, dtype=np.uint32)
    b = rng.integers(0, 2**32, 128, dtype=np.uint32)
    truth = int((a.astype(np.uint64) * b.astype(np.uint64) % 2**32).sum() % 2**32)
    assert oracle.inner_product(a, b) == truth


def ip_closed_form(N, D=128):
    return (D * (D - 1) // 2 * N * (N - 1) // 2 + (D - 1) * D * (2 * D - 1) // 6 * N) % 2**32


def test_inner_product_bench_closed_form(oracle):
    # graphann_test.go:249-283 fill; SURVEY §8a a2 golden 1,178,525,696 at N=1e8
    assert ip_closed_form(100_000_000) == 1_178_525_696
    for N in (1, 2, 1000, 123457):
        assert oracle.inner_product_bench(N, 128, 4) == ip_closed_form(N)


def l2_numpy_asm_order(a, b):
    f = np.float32
    n = len(a) & ~7
    s = np.zeros(8, np.float32)
    for t in range(0, n, 8):
        d = (a[t:t + 8] - b[t:t + 8]).astype(np.float32)
        s = (s + d * d).astype(np.float32)
    r = f(f(f(s[0] + s[1]) + f(s[2] + s[3])) + f(f(s[4] + s[5]) + f(s[6] + s[7]))) if n else f(0)
    for i in range(n, len(a)):
        d = f(a[i] - b[i])
        r = f(r + f(d * d))
    return r


@pytest.mark.parametrize("dim", [8, 128, 192, 13, 3])
def test_l2_order(oracle, dim):
    rng = np.random.default_rng(dim)
    for _ in range(50):
        a = (rng.standard_normal(dim) * 100).astype(np.float32)
        b = (rng.standard_normal(dim) * 100).astype(np.float32)
        want = l2_numpy_asm_order(a, b)
        assert np.float32(oracle.l2dist(a, b)).view(np.uint32) == want.view(np.uint32)
        if dim % 8 == 0:   # the AVX-intrinsic restatement of the asm agrees too
            assert np.float32(oracle.l2dist_avx(a, b)).view(np.uint32) == want.view(np.uint32)


def test_l2_msmarco_golden(oracle):
    g = load_golden("l2_msmarco")
    for i, q in enumerate(g["queries"]):
        assert np.array_equal(oracle.l2_batch(q, g["documents"]).view(np.uint32), g["dist"][i].view(np.uint32))


# --- parameters & accounting (private-search-report.txt, msmarco README) ----
def _batch(oracle, N, E, B=32, F=8):
    db = np.zeros(1, np.uint64)   # never read before Preprocessing
    return oracle.SimpleBatchPianoPIR(N, E * 8, B, np.zeros(N * E, np.uint64) if N * E < 2**27 else db, F)


def test_sift1m_parameters_match_report(oracle):
    """private-search-report.txt:5-21 for SIFT1M n=1e6, d=128, m=32, step 20, parallel 3."""
    N, E = 1_000_000, 80
    db = np.zeros(N * E, np.uint64)
    b = oracle.SimpleBatchPianoPIR(N, E * 8, 32, db, 8)
    b.DummyPreprocessing()
    s = b.stats()
    sub = b.sub(0).Config()
    assert (sub["ChunkSize"], sub["SetSize"], sub["MaxQueryNum"], sub["PrimaryHintNum"],
            sub["MaxQueryPerChunk"]) == (512, 124, 2760, 3584, 72)
    assert s["SupportBatchNum"] == 1380
    assert s["SupportBatchNum"] // (20 * 3) == 23                                   # Window Size
    assert f"{N * 640 / 1024 / 1024:f}" == "610.351562"                              # DB Size (MB)
    assert f"{s['LocalStorage'] / 1024 / 1024:f}" == "212.429688"                    # Storage (MB)
    assert f"{s['CommOffline'] * 20 * 3 / 1024:f}" == "27173.906250"                # Offline comm / Q
    assert f"{s['CommOnline'] * 20 * 3 / 1024:f}" == "2130.000000"                  # Online comm / Q


def test_msmarco_parameters(oracle):
    """reproduction/msmarco/README.md:261-265: 3,150 KB online comm per query."""
    N, E = 3_201_821, 112
    b = oracle.SimpleBatchPianoPIR(N, E * 8, 32, np.zeros(N * E, np.uint64), 8)
    b.DummyPreprocessing()
    s = b.stats()
    sub = b.sub(0).Config()
    assert (sub["ChunkSize"], sub["SetSize"], sub["MaxQueryNum"], sub["PrimaryHintNum"],
            sub["MaxQueryPerChunk"]) == (1024, 196, 5460, 7168, 88)
    assert round(s["CommOnline"] * 60 / 1024) == 3150
    assert s["SupportBatchNum"] // 60 == 45


def test_oracle_robust_prune_properties():
    """robustPrune (build_graph.go:169-236) restated: lists of at most m come
    back unchanged; otherwise exactly m ids, the nearest candidate first, and
    with alpha = 0 (no candidate ever dominated) the m nearest in order."""
    import numpy as np
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    X = rng.integers(0, 256, size=(200, 16)).astype(np.float32)
    cand = np.arange(1, 41, dtype=np.uint32)
    assert np.array_equal(O.robust_prune(X, 0, cand[:8], 8), cand[:8])
    r = O.robust_prune(X, 0, cand, 8, 1.2)
    d = O.l2_batch(X[0], X[cand])
    assert len(r) == 8 and r[0] == cand[np.argmin(d)]
    r0 = O.robust_prune(X, 0, cand, 8, 0.0)
    assert np.array_equal(r0, cand[np.lexsort((np.arange(40), d))][:8])


def test_oracle_build_graph_properties():
    """The graph restatement: m neighbours per row, no self loops, deterministic
    in the seed, different across seeds (sampling and fill).  A row may repeat
    an id, as the reference's may: a mutual edge appears twice in biGraph and
    both copies can survive sampling when the list is not pruned (:445-462)."""
    import numpy as np
    from oracle import oracle as O
    from tests.datagen import clustered_vectors
    v = clustered_vectors(600, 32, seed=1)
    g = O.build_graph(v, 12, 1.2, seed=4)
    assert g.shape == (600, 12)
    assert (g != np.arange(600)[:, None]).all()
    assert np.array_equal(g, O.build_graph(v, 12, 1.2, seed=4))
    assert not np.array_equal(g, O.build_graph(v, 12, 1.2, seed=5))
    ids, _ = O.knn(v, v[:3], 5)
    assert (ids[:, 0] == np.arange(3)).all()   # each row's own nearest is itself
