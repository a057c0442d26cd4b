"""Generate the committed golden fixtures (run here, where /root/reference exists).

    python tests/golden/make_golden.py

Fixtures are data only (inputs + expected outputs):
  l2_msmarco.npz   real d=192 MS-MARCO vectors from the reference's own fixture
                   reproduction/msmarco/assets/validation_reference.npz
                   (reduced_queries[:16], reduced_documents), float64 -> float32 as
                   graphann/loader.go:190 does, with L2Dist in the asm's order
                   (l2_distance_amd64.s:4-36), computed independently in numpy.
  prf_vectors.json AES-128-MMO PRF vectors (util.go:157-165) computed with OpenSSL's
                   AES_encrypt (independent of both the oracle and the product).
  pir_transcript.npz / batch_transcript.npz
                   oracle transcripts (responses + state digests) on seeded DBs;
                   they pin the oracle against regressions and travel to the GPU box.
"""
import ctypes as C
import hashlib
import json
import struct
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT))
REF_NPZ = Path("/root/reference/reproduction/msmarco/assets/validation_reference.npz")


def l2_asm_order(a, b):
    """numpy restatement of L2DistanceSIMD + L2Dist tail, float32 throughout."""
    a = a.astype(np.float32)
    b = b.astype(np.float32)
    n = len(a) & ~7
    s = np.zeros(8, np.float32)
    for t in range(0, n, 8):
        d = (a[t:t + 8] - b[t:t + 8]).astype(np.float32)
        s = (s + (d * d).astype(np.float32)).astype(np.float32)
    f = np.float32
    r = f(f(f(s[0] + s[1]) + f(s[2] + s[3])) + f(f(s[4] + s[5]) + f(s[6] + s[7]))) if n else f(0)
    for i in range(n, len(a)):
        d = f(a[i] - b[i])
        r = f(r + f(d * d))
    return r


def openssl_prf(key: bytes, tag: int, x: int) -> int:
    crypto = C.CDLL("libcrypto.so.3")
    aes_key = C.create_string_buffer(244)
    assert crypto.AES_set_encrypt_key(key, 128, aes_key) == 0
    blk = struct.pack("<Q", ((tag << 35) + x) & (2**64 - 1)) + bytes(8)
    out = C.create_string_buffer(16)
    crypto.AES_encrypt(blk, out, aes_key)
    c = bytes(p ^ q for p, q in zip(out.raw, blk))
    return struct.unpack("<Q", c[:8])[0]


def main():
    from oracle import oracle as O

    # --- L2 on real MS-MARCO vectors --------------------------------------
    with np.load(REF_NPZ, allow_pickle=False) as z:
        qs = z["reduced_queries"][:16].astype(np.float32)
        docs = z["reduced_documents"].astype(np.float32)
    dist = np.array([[l2_asm_order(d, q) for d in docs] for q in qs], np.float32)
    for i, q in enumerate(qs):
        assert np.array_equal(O.l2_batch(q, docs).view(np.uint32), dist[i].view(np.uint32))
    np.savez_compressed(HERE / "l2_msmarco.npz", queries=qs, documents=docs, dist=dist)

    # --- PRF vectors via OpenSSL -----------------------------------------
    rng = np.random.default_rng(2024)
    keys = [bytes(range(16))] + [rng.bytes(16) for _ in range(7)]
    vec = []
    for k in keys:
        tags = [0, 1, 5, 3583, 12511, (1 << 29) - 1] + [int(t) for t in rng.integers(0, 2**29, 10)]
        xs = [0, 7, 123, 3815, 2**35 - 1] + [int(t) for t in rng.integers(0, 2**35, 11)]
        rk = O.expand_key(k)
        for t, x in zip(tags, xs):
            want = openssl_prf(k, t, x)
            assert O.prf(rk, t, x) == want
            vec.append({"key": k.hex(), "tag": t, "x": x, "prf": f"{want:016x}"})
    (HERE / "prf_vectors.json").write_text(json.dumps({"source": "OpenSSL AES_encrypt", "vectors": vec}, indent=0))

    # --- oracle transcripts ----------------------------------------------
    N, E, F, seed = 3000, 4, 8, 77
    db = np.random.default_rng(1).integers(0, 2**64, size=N * E, dtype=np.uint64)
    p = O.PianoPIR(N, E * 8, db, F, seed=seed)
    p.Preprocessing()
    ids = np.random.default_rng(2).integers(0, N, size=300)
    resp, st = [], []
    for i in ids:
        r, s = p.Query(int(i), True)
        resp.append(r)
        st.append(s)
    state = p.export_state()
    dig = hashlib.sha256(b"".join(state[k].tobytes() for k in sorted(state))).hexdigest()
    np.savez_compressed(HERE / "pir_transcript.npz", N=N, E=E, F=F, seed=seed, db_seed=1, ids=ids,
                        responses=np.array(resp), status=np.array(st), state_sha256=np.array(dig))

    N, E, B = 20000, 12, 32
    db = np.random.default_rng(3).integers(0, 2**64, size=N * E, dtype=np.uint64)
    b = O.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=seed)
    b.Preprocessing()
    batches = np.random.default_rng(4).integers(0, N, size=(40, 96)).astype(np.uint64)
    out = np.array([b.Query(q)[0] for q in batches])
    np.savez_compressed(HERE / "batch_transcript.npz", N=N, E=E, B=B, F=8, seed=seed, db_seed=3,
                        batches=batches, responses=out)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
