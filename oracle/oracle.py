"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see pm_oracle.h).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  The product (pacmann_amd / libpacmann.so) never does.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"
_lib = None

vp, u64 = C.c_void_p, C.c_uint64
u32p, u64p, i64p, f32p = (C.POINTER(C.c_uint32), C.POINTER(C.c_uint64), C.POINTER(C.c_int64),
                          C.POINTER(C.c_float))


class OrPirConfig(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "DBEntryByteNum DBEntrySize DBSize ChunkSize SetSize ThreadNum FailureProbLog2 "
        "MaxQueryNum PrimaryHintNum MaxQueryPerChunk FinishedQueryNum").split()]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class OrBatchStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "DBEntryByteNum DBEntrySize DBSize BatchSize PartitionNum PartitionSize ThreadNum "
        "FailureProbLog2 FinishedBatchNum QueriesMadeInPartition SupportBatchNum PrepCount").split()] + \
        [(n, C.c_double) for n in "LocalStorage PreprocessingTime CommOnline CommOffline".split()]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


SIG = {
    "or_expand_key": (None, [C.c_char_p, u32p]),
    "or_aes128_encrypt": (None, [u32p, C.c_char_p, C.c_char_p]),
    "or_prf": (u64, [u32p, u64, u64]),
    "or_prf_batch": (None, [u32p, u64p, u64p, u64, u64p]),
    "or_xor_slices": (None, [u64p, u64p, u64]),
    "or_derive_key": (None, [u64, u64, u64, C.c_char_p]),
    "or_hash4": (u64, [u64, u64, u64, u64, u64]),
    "or_l2dist": (C.c_float, [f32p, f32p, u64]),
    "or_l2dist_avx": (C.c_float, [f32p, f32p, u64]),
    "or_inner_product": (C.c_uint32, [u32p, u32p, u64]),
    "or_inner_product_bench": (C.c_uint32, [u64, u64, C.c_int]),
    "or_inner_product_scan": (C.c_uint32, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), u64, u64, C.c_int]),
    "or_l2_batch": (None, [f32p, f32p, u64, u64, f32p]),
    "or_set_prep_threads": (None, [C.c_int]),
    "or_pir_new": (vp, [u64, u64, u64p, u64, u64, u64]),
    "or_pir_free": (None, [vp]),
    "or_pir_preprocessing": (None, [vp]),
    "or_pir_dummy_preprocessing": (None, [vp]),
    "or_pir_query": (C.c_int, [vp, u64, C.c_int, u64p]),
    "or_server_private_query": (C.c_int, [vp, u32p, u64p]),
    "or_pir_config_get": (None, [vp, C.POINTER(OrPirConfig)]),
    "or_pir_local_storage": (C.c_double, [vp]),
    "or_pir_comm_per_query": (C.c_double, [vp]),
    "or_pir_epoch": (u64, [vp]),
    "or_pir_export": (None, [vp, u32p, u64p, u64p, u64p, u64p, u64p, u64p, u64p, u64p]),
    "or_batch_new": (vp, [u64, u64, u64, u64p, u64, u64]),
    "or_batch_free": (None, [vp]),
    "or_batch_preprocessing": (None, [vp]),
    "or_batch_dummy_preprocessing": (None, [vp]),
    "or_batch_query": (C.c_int, [vp, u64p, u64, u64p]),
    "or_batch_stats_get": (None, [vp, C.POINTER(OrBatchStats)]),
    "or_batch_subpir": (vp, [vp, u64]),
    "or_graph_new": (vp, [u64, u64, u64, f32p, u32p, C.c_int, C.c_int, u64, u64]),
    "or_graph_free": (None, [vp]),
    "or_graph_preprocess": (None, [vp]),
    "or_search_knn": (None, [vp, f32p, C.c_int, C.c_int, C.c_int, C.c_int, i64p, i64p]),
    "or_graph_counts": (None, [vp, u64p, u64p]),
    "or_graph_pir": (vp, [vp]),
    "or_knn": (None, [f32p, u64, u64, f32p, u64, C.c_uint32, i64p, f32p]),
    "or_robust_prune": (None, [f32p, u64, u64, u32p, u64, u64, C.c_float, u32p, C.POINTER(C.c_uint32)]),
    "or_build_graph": (C.c_int, [f32p, u64, u64, u64, C.c_float, u64, u32p]),
    "or_search_loop": (None, [vp, f32p, u64, C.c_int, C.c_int, C.c_int, C.c_int, i64p,
                              C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "or_graph_get_vertex_info": (None, [vp, i64p, u64, f32p, u32p]),
    "or_graph_get_start_vertex": (u64, [vp, u64, i64p, f32p, u32p]),
}


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
        L = C.CDLL(str(LIB_PATH))
        for n, (r, a) in SIG.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def set_prep_threads(n: int) -> None:
    """Threads of the hint fold in Preprocessing (1 = the reference's loop).
    They split the hint space, so the client state is identical for any n."""
    lib().or_set_prep_threads(int(n))


def _p(a, t):
    return a.ctypes.data_as(t)


def expand_key(key: bytes) -> np.ndarray:
    rk = np.zeros(44, np.uint32)
    lib().or_expand_key(bytes(key), _p(rk, u32p))
    return rk


def aes128_encrypt(rk, block: bytes) -> bytes:
    out = C.create_string_buffer(16)
    lib().or_aes128_encrypt(_p(np.ascontiguousarray(rk, np.uint32), u32p), bytes(block), out)
    return out.raw


def prf(rk, tag: int, x: int) -> int:
    return lib().or_prf(_p(np.ascontiguousarray(rk, np.uint32), u32p), tag, x)


def prf_batch(rk, tags, xs) -> np.ndarray:
    t = np.ascontiguousarray(tags, np.uint64)
    x = np.ascontiguousarray(xs, np.uint64)
    out = np.zeros(len(t), np.uint64)
    lib().or_prf_batch(_p(np.ascontiguousarray(rk, np.uint32), u32p), _p(t, u64p), _p(x, u64p),
                       len(t), _p(out, u64p))
    return out


def derive_key(seed: int, partition: int, epoch: int) -> bytes:
    k = C.create_string_buffer(16)
    lib().or_derive_key(seed, partition, epoch, k)
    return k.raw


def xor_slices(dst: np.ndarray, src: np.ndarray):
    lib().or_xor_slices(_p(dst, u64p), _p(src, u64p), len(src))


def l2dist(a, b) -> float:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return lib().or_l2dist(_p(a, f32p), _p(b, f32p), len(a))


def l2dist_avx(a, b) -> float:
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return lib().or_l2dist_avx(_p(a, f32p), _p(b, f32p), len(a))


def l2_batch(q, rows) -> np.ndarray:
    q = np.ascontiguousarray(q, np.float32)
    r = np.ascontiguousarray(rows, np.float32).reshape(-1, len(q))
    out = np.zeros(r.shape[0], np.float32)
    lib().or_l2_batch(_p(q, f32p), _p(r, f32p), r.shape[0], len(q), _p(out, f32p))
    return out


def inner_product(a, b) -> int:
    a = np.ascontiguousarray(a, np.uint32)
    b = np.ascontiguousarray(b, np.uint32)
    return lib().or_inner_product(_p(a, u32p), _p(b, u32p), len(a))


def inner_product_bench(N: int, D: int, nthreads: int = 1) -> int:
    return lib().or_inner_product_bench(N, D, nthreads)


def inner_product_scan(rows: np.ndarray, q: np.ndarray, nthreads: int = 1) -> int:
    """InnerProduct summed over materialised rows (N x D uint32), mod 2^32."""
    rows = np.ascontiguousarray(rows, np.uint32)
    q = np.ascontiguousarray(q, np.uint32)
    return lib().or_inner_product_scan(_p(rows, C.POINTER(C.c_uint32)), _p(q, C.POINTER(C.c_uint32)),
                                       rows.shape[0], rows.shape[1], nthreads)


def _export(h, cfg: dict) -> dict:
    E, PH, SS, Q = cfg["DBEntrySize"], cfg["PrimaryHintNum"], cfg["SetSize"], cfg["MaxQueryPerChunk"]
    nb = SS * Q
    st = {
        "round_keys": np.zeros(44, np.uint32),
        "primary_tag": np.zeros(PH, np.uint64), "primary_parity": np.zeros(PH * E, np.uint64),
        "primary_pp": np.zeros(PH, np.uint64), "backup_tag": np.zeros(nb, np.uint64),
        "backup_parity": np.zeros(nb * E, np.uint64), "repl_idx": np.zeros(nb, np.uint64),
        "repl_val": np.zeros(nb * E, np.uint64), "hist": np.zeros(SS, np.uint64),
    }
    lib().or_pir_export(h, _p(st["round_keys"], u32p), *[_p(st[k], u64p) for k in (
        "primary_tag", "primary_parity", "primary_pp", "backup_tag", "backup_parity", "repl_idx",
        "repl_val", "hist")])
    return st


class PianoPIR:
    def __init__(self, DBSize, DBEntryByteNum, rawDB, FailureProbLog2, seed=1, partition=0,
                 _handle=None, _keep=None):
        if _handle is not None:
            self.h, self._owned, self._db = _handle, False, _keep
        else:
            self._db = np.ascontiguousarray(rawDB, np.uint64)   # the oracle aliases it (pir.go:34-39)
            self.h = lib().or_pir_new(DBSize, DBEntryByteNum, _p(self._db, u64p), FailureProbLog2, seed,
                                      partition)
            self._owned = True
        self.E = self.Config()["DBEntrySize"]

    def __del__(self):
        if getattr(self, "_owned", False) and self.h:
            lib().or_pir_free(self.h)
            self.h = None

    def Preprocessing(self):
        lib().or_pir_preprocessing(self.h)

    def DummyPreprocessing(self):
        lib().or_pir_dummy_preprocessing(self.h)

    def Query(self, idx, realQuery=True):
        out = np.zeros(self.E, np.uint64)
        st = lib().or_pir_query(self.h, idx, int(realQuery), _p(out, u64p))
        return out, st

    def PrivateQuery(self, offsets):
        o = np.ascontiguousarray(offsets, np.uint32)
        out = np.zeros(self.E, np.uint64)
        lib().or_server_private_query(self.h, _p(o, u32p), _p(out, u64p))
        return out

    def Config(self):
        c = OrPirConfig()
        lib().or_pir_config_get(self.h, C.byref(c))
        return c.asdict()

    def LocalStorageSize(self):
        return lib().or_pir_local_storage(self.h)

    def CommCostPerQuery(self):
        return lib().or_pir_comm_per_query(self.h)

    def export_state(self):
        return _export(self.h, self.Config())


class SimpleBatchPianoPIR:
    def __init__(self, DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2, seed=1,
                 _handle=None, _keep=None):
        if _handle is not None:
            self.h, self._owned, self._db = _handle, False, _keep
        else:
            self._db = np.ascontiguousarray(rawDB, np.uint64)
            self.h = lib().or_batch_new(DBSize, DBEntryByteNum, BatchSize, _p(self._db, u64p),
                                        FailureProbLog2, seed)
            self._owned = True
        self.E = self.stats()["DBEntrySize"]

    def __del__(self):
        if getattr(self, "_owned", False) and self.h:
            lib().or_batch_free(self.h)
            self.h = None

    def Preprocessing(self):
        lib().or_batch_preprocessing(self.h)

    def DummyPreprocessing(self):
        lib().or_batch_dummy_preprocessing(self.h)

    def Query(self, idx):
        ids = np.ascontiguousarray(idx, np.uint64).ravel()
        out = np.zeros((len(ids), self.E), np.uint64)
        rc = lib().or_batch_query(self.h, _p(ids, u64p), len(ids), _p(out, u64p))
        return out, (None if rc == 0 else rc)

    def stats(self):
        s = OrBatchStats()
        lib().or_batch_stats_get(self.h, C.byref(s))
        return s.asdict()

    def sub(self, i) -> PianoPIR:
        return PianoPIR(0, 0, None, 0, _handle=lib().or_batch_subpir(self.h, i), _keep=self._db)


class Graph:
    def __init__(self, vectors, graph, nonprivate=False, skip_prep=False, pir_seed=1, search_seed=1):
        self._v = np.ascontiguousarray(vectors, np.float32)
        self._g = np.ascontiguousarray(graph, np.uint32)
        self.N, self.Dim = self._v.shape
        self.M = self._g.shape[1]
        self.h = lib().or_graph_new(self.N, self.Dim, self.M, _p(self._v, f32p), _p(self._g, u32p),
                                    int(nonprivate), int(skip_prep), pir_seed, search_seed)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_graph_free(self.h)
            self.h = None

    def Preprocess(self):
        lib().or_graph_preprocess(self.h)

    def SearchKNN(self, q, k, maxStep, parallel, benchmarking=False):
        q = np.ascontiguousarray(q, np.float32)
        ids = np.zeros(k, np.int64)
        steps = np.zeros(k, np.int64)
        lib().or_search_knn(self.h, _p(q, f32p), k, maxStep, parallel, int(benchmarking), _p(ids, i64p),
                            _p(steps, i64p))
        return ids, steps

    def SearchLoop(self, queries, k, step, parallel, benchmarking=False):
        qs = np.ascontiguousarray(queries, np.float32)
        ans = np.zeros((qs.shape[0], k), np.int64)
        on, mt = C.c_double(), C.c_double()
        lib().or_search_loop(self.h, _p(qs, f32p), qs.shape[0], k, step, parallel, int(benchmarking),
                             _p(ans, i64p), C.byref(on), C.byref(mt))
        return ans, on.value, mt.value

    def counts(self):
        t, s = C.c_uint64(), C.c_uint64()
        lib().or_graph_counts(self.h, C.byref(t), C.byref(s))
        return t.value, s.value

    def GetMetadata(self):
        return self.N, self.Dim, self.M

    def GetVertexInfo(self, ids):
        """PIRGraphInfo.GetVertexInfo (private-search.go:441-506): (vectors [n, dim], neighbours [n, m])."""
        i = np.ascontiguousarray(ids, np.int64).ravel()
        vec = np.zeros((len(i), self.Dim), np.float32)
        nb = np.zeros((len(i), self.M), np.uint32)
        lib().or_graph_get_vertex_info(self.h, _p(i, i64p), len(i), _p(vec, f32p), _p(nb, u32p))
        return vec, nb

    def GetStartVertex(self):
        """PIRGraphInfo.GetStartVertex (private-search.go:508-531): (ids, vectors, neighbours)."""
        n = int(lib().or_graph_get_start_vertex(self.h, 0, None, None, None))
        ids = np.zeros(n, np.int64)
        vec = np.zeros((n, self.Dim), np.float32)
        nb = np.zeros((n, self.M), np.uint32)
        lib().or_graph_get_start_vertex(self.h, n, _p(ids, i64p), _p(vec, f32p), _p(nb, u32p))
        return ids, vec, nb

    def pir(self) -> SimpleBatchPianoPIR:
        return SimpleBatchPianoPIR(0, 0, 0, None, 0, _handle=lib().or_graph_pir(self.h), _keep=self._v)


def knn(base, queries, k):
    """Exact (L2Dist, id) top k by brute force (or_knn)."""
    b = np.ascontiguousarray(base, dtype=np.float32)
    q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, b.shape[1])
    ids = np.zeros((q.shape[0], k), dtype=np.int64)
    d = np.zeros((q.shape[0], k), dtype=np.float32)
    lib().or_knn(_p(b, f32p), b.shape[0], b.shape[1], _p(q, f32p), q.shape[0], k, _p(ids, i64p),
                 _p(d, f32p))
    return ids, d


def robust_prune(X, u, cand, m, alpha=1.2):
    X = np.ascontiguousarray(X, dtype=np.float32)
    c = np.ascontiguousarray(cand, dtype=np.uint32)
    out = np.zeros(max(len(c), m), dtype=np.uint32)
    n = C.c_uint32()
    lib().or_robust_prune(_p(X, f32p), X.shape[1], u, _p(c, u32p), len(c), m, C.c_float(alpha),
                          _p(out, u32p), C.byref(n))
    return out[:n.value]


def build_graph(X, m, alpha=1.2, seed=1):
    X = np.ascontiguousarray(X, dtype=np.float32)
    g = np.zeros((X.shape[0], m), dtype=np.uint32)
    rc = lib().or_build_graph(_p(X, f32p), X.shape[0], X.shape[1], m, C.c_float(alpha), seed, _p(g, u32p))
    if rc:
        raise ValueError("or_build_graph: n must be > m")
    return g
