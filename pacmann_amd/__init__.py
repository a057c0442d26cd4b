"""pacmann_amd — MI355X-native PianoPIR + graphann hot path (libpacmann.so).

Python mirror of the reference's Go package surfaces, bound through the C ABI
in include/pacmann.h.  Names, argument meaning and error behaviour follow the
reference so that tests read like pianopir/pir_test.go:

    pir = SimpleBatchPianoPIR(DBSize, DBEntryByteNum, BatchSize, rawDB, FailureProbLog2)
    pir.Preprocessing()
    responses, err = pir.Query(batch)

There is no CPU fallback: constructing any handle without a built
libpacmann.so or without a HIP device raises.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

__all__ = [
    "Context", "PianoPIR", "SimpleBatchPianoPIR", "PIRGraphInfo", "GraphANNFrontend",
    "lib", "expand_key", "prf_batch", "l2_batch", "ip_batch", "ip_bench", "LIB_PATH",
    "QueryError",
]

import os as _os

# PM_LIB selects a diagnostic build (e.g. the PM_STAMPS variant); default is the product .so
LIB_PATH = Path(_os.environ.get("PM_LIB") or (Path(__file__).resolve().parent / "libpacmann.so"))
_lib = None

u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)
f32p = C.POINTER(C.c_float)
vp = C.c_void_p
u64 = C.c_uint64
dbl = C.c_double


class PirConfig(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "DBEntryByteNum DBEntrySize DBSize ChunkSize SetSize ThreadNum FailureProbLog2 "
        "MaxQueryNum PrimaryHintNum MaxQueryPerChunk FinishedQueryNum").split()]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class BatchStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in (
        "DBEntryByteNum DBEntrySize DBSize BatchSize PartitionNum PartitionSize ThreadNum "
        "FailureProbLog2 FinishedBatchNum QueriesMadeInPartition SupportBatchNum PrepCount").split()] + \
        [(n, C.c_double) for n in "LocalStorage PreprocessingTime CommOnline CommOffline".split()]

    def asdict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


# pm_combine_fn (include/pacmann.h): (user, team, dev_words, nwords, stream) -> 0 on success
COMBINE_FN = C.CFUNCTYPE(C.c_int, vp, C.c_uint32, vp, u64, vp)

# name -> (restype, argtypes) ; every exported symbol of include/pacmann.h
SIGNATURES = {
    "pm_ctx_create": (C.c_int, [C.c_int, C.POINTER(vp)]),
    "pm_ctx_destroy": (None, [vp]),
    "pm_last_error": (C.c_char_p, []),
    "pm_ctx_sync": (C.c_int, [vp]),
    "pm_ctx_mem_info": (C.c_int, [vp, u64p, u64p]),
    "pm_timing_enable": (C.c_int, [vp, C.c_int]),
    "pm_set_option": (C.c_int, [C.c_char_p, C.c_int]),
    "pm_timing_reset": (C.c_int, [vp]),
    "pm_timing_get": (C.c_int, [vp, C.c_char_p, u64p, C.POINTER(dbl), C.POINTER(dbl)]),
    "pm_timing_timeline": (C.c_int, [vp, C.c_char_p]),
    "pm_expand_key": (C.c_int, [u8p, u32p]),
    "pm_prf_batch": (C.c_int, [vp, u32p, u64p, u64p, u64, u64p]),
    "pm_l2_batch": (C.c_int, [vp, f32p, f32p, u64, u64, f32p]),
    "pm_ip_batch": (C.c_int, [vp, u32p, u32p, u64, u64, u32p, u32p]),
    "pm_ip_bench": (C.c_int, [vp, u64, u64, u32p, C.POINTER(dbl)]),
    "pm_ip_bench_shard": (C.c_int, [vp, u64, u64, u64, u64, u32p, C.POINTER(dbl)]),
    "pm_pir_create": (C.c_int, [vp, u64, u64, u64p, u64, u64, C.POINTER(vp)]),
    "pm_pir_destroy": (None, [vp]),
    "pm_pir_preprocessing": (C.c_int, [vp]),
    "pm_pir_dummy_preprocessing": (C.c_int, [vp]),
    "pm_pir_query": (C.c_int, [vp, u64, C.c_int, u64p, C.POINTER(C.c_int)]),
    "pm_pir_config_get": (C.c_int, [vp, C.POINTER(PirConfig)]),
    "pm_pir_local_storage": (C.c_double, [vp]),
    "pm_pir_comm_per_query": (C.c_double, [vp]),
    "pm_pir_server_answer": (C.c_int, [vp, u32p, u64, u64p]),
    "pm_batchpir_create": (C.c_int, [vp, u64, u64, u64, u64p, u64, u64, C.POINTER(vp)]),
    "pm_batchpir_destroy": (None, [vp]),
    "pm_batchpir_preprocessing": (C.c_int, [vp]),
    "pm_batchpir_dummy_preprocessing": (C.c_int, [vp]),
    "pm_batchpir_query": (C.c_int, [vp, u64p, u64, u64p]),
    "pm_batchpir_query_ok": (C.c_int, [vp, u64p, u64, u64p, C.POINTER(C.c_uint8)]),
    "pm_batchpir_query_dev": (C.c_int, [vp, u64p, u64, vp, vp]),
    "pm_batchpir_create_shard": (C.c_int, [vp, u64, u64, u64, u64p, u64, u64, C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "pm_batchpir_create_synth": (C.c_int, [vp, u64, u64, u64, u64, u64, u64, C.c_uint32, C.c_uint32, C.POINTER(vp)]),
    "pm_batchpir_stats_get": (C.c_int, [vp, C.POINTER(BatchStats)]),
    "pm_batchpir_subconfig": (C.c_int, [vp, u64, C.POINTER(PirConfig)]),
    "pm_pir_export": (C.c_int, [vp, u32p, u64p, u64p, u64p, u64p, u64p, u64p, u64p, u64p]),
    "pm_batchpir_export": (C.c_int, [vp, u64, u32p, u64p, u64p, u64p, u64p, u64p, u64p, u64p, u64p]),
    "pm_graph_create": (C.c_int, [vp, u64, u64, u64, f32p, u32p, C.c_int, C.c_int, u64, u64, C.POINTER(vp)]),
    "pm_graph_destroy": (None, [vp]),
    "pm_graph_preprocess": (C.c_int, [vp]),
    "pm_search_knn": (C.c_int, [vp, f32p, C.c_int, C.c_int, C.c_int, C.c_int, i64p, i64p]),
    "pm_search_loop": (C.c_int, [vp, f32p, u64, C.c_int, C.c_int, C.c_int, C.c_int, i64p,
                                 C.POINTER(dbl), C.POINTER(dbl)]),
    "pm_graph_counts": (C.c_int, [vp, u64p, u64p]),
    "pm_graph_pir": (vp, [vp]),
    "pm_batchpir_create_client": (C.c_int, [vp, vp, u64, C.POINTER(vp)]),
    "pm_graph_create_session": (C.c_int, [vp, vp, u64, u64, C.POINTER(vp)]),
    "pm_knn": (C.c_int, [vp, f32p, u64, u64, f32p, u64, C.c_uint32, i64p, f32p]),
    "pm_build_graph": (C.c_int, [vp, f32p, u64, u64, u64, C.c_float, u64, u32p, C.POINTER(dbl)]),
    "pm_search_loop_sessions": (C.c_int, [C.POINTER(vp), C.c_uint32, f32p, u64, C.c_int, C.c_int, C.c_int,
                                          i64p, C.POINTER(dbl), C.POINTER(dbl), C.POINTER(dbl)]),
    "pm_batchpir_group_create": (C.c_int, [C.POINTER(vp), C.c_uint32, C.POINTER(vp)]),
    "pm_batchpir_group_query": (C.c_int, [vp, u64p, u64, u64p, C.POINTER(C.c_uint8)]),
    "pm_batchpir_group_preprocessing": (C.c_int, [vp]),
    "pm_batchpir_group_destroy": (None, [vp]),
    "pm_search_loop_batched": (C.c_int, [C.POINTER(vp), C.c_uint32, f32p, u64, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                         C.c_uint32, i64p, C.POINTER(dbl), C.POINTER(dbl), C.POINTER(dbl)]),
    "pm_graph_create_shard": (C.c_int, [vp, u64, u64, u64, f32p, u32p, C.c_uint32, C.c_uint32, u64, u64,
                                        C.POINTER(vp)]),
    "pm_graph_create_synth": (C.c_int, [vp, u64, u64, u64, u64, C.c_uint32, C.c_uint32, u64, u64, C.POINTER(vp)]),
    "pm_graph_synth_rows": (C.c_int, [u64, u64, u64, u64, u64p, u64, f32p, u32p]),
    "pm_sharded_record_words": (u64, [vp, C.c_uint32, C.c_int]),
    "pm_search_loop_sharded": (C.c_int, [C.POINTER(vp), C.c_uint32, f32p, u64, C.c_int, C.c_int, C.c_int, C.c_uint32,
                                         C.c_uint32, COMBINE_FN, vp, C.POINTER(vp), C.c_int, i64p, C.POINTER(dbl),
                                         C.POINTER(dbl), C.POINTER(dbl)]),
    "pm_graph_get_metadata": (C.c_int, [vp, u64p, u64p, u64p]),
    "pm_graph_get_vertex_info": (C.c_int, [vp, u64p, u64, f32p, u32p, u8p, f32p, f32p]),
    "pm_graph_get_start_vertex": (C.c_int, [vp, u64, u64p, f32p, u32p, u64p]),
    "pm_rccl_unique_id": (C.c_int, [u8p]),
    "pm_rccl_create": (C.c_int, [C.c_int, C.c_int, C.c_int, u8p, C.c_uint32, C.POINTER(vp)]),
    "pm_rccl_destroy": (None, [vp]),
    "pm_rccl_combine": (C.c_int, [vp, C.c_uint32, vp, u64, vp]),
    "pm_rccl_probe": (C.c_int, [vp]),
}
RCCL_ID_BYTES = 128   # PM_RCCL_ID_BYTES

Q_OK, Q_EBUDGET, Q_ECHUNK, Q_ENOHIT, Q_ERANGE = range(5)
_QERR = {
    Q_EBUDGET: "exceed the maximum number of queries",
    Q_ECHUNK: "too many queries in chunk",
    Q_ENOHIT: "no hit hint in the primary hint table",
    Q_ERANGE: "idx is out of range",
}


class QueryError(Exception):
    """Recoverable per-query error (the reference's `error` return value)."""

    def __init__(self, code: int):
        super().__init__(_QERR.get(code, f"status {code}"))
        self.code = code


def lib() -> C.CDLL:
    """Load libpacmann.so; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: run `python -m pacmann_amd.build` "
                               "(there is no CPU fallback)")
        L = C.CDLL(str(LIB_PATH))
        for name, (res, args) in SIGNATURES.items():
            if _os.environ.get("PM_LIB") and not hasattr(L, name):
                continue   # an older diagnostic build (A/B runs): its missing entry points stay unbound
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def hip_runtimes() -> set[str]:
    """Paths of the HIP runtime libraries mapped into this process.  torch's
    ROCm wheel ships its own libamdhip64 (same SONAME as /opt/rocm's): with
    torch imported first, libpacmann.so binds to that one copy; loading
    libpacmann.so first and torch later maps a second runtime, whose streams
    and events the first cannot use (pacmann_amd.shard refuses that case)."""
    with open("/proc/self/maps") as fh:
        return {ln.split()[-1] for ln in fh if "libamdhip64" in ln}


def _check(rc: int):
    if rc != 0:
        raise RuntimeError(f"libpacmann error {rc}: {lib().pm_last_error().decode()}")


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def _u64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint64))


class Context:
    """One HIP device + stream (pm_ctx)."""

    def __init__(self, device: int = 0):
        h = vp()
        _check(lib().pm_ctx_create(device, C.byref(h)))
        self.h = h
        self.device = device

    def close(self):
        if getattr(self, "h", None):
            lib().pm_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        _check(lib().pm_ctx_sync(self.h))

    def mem_info(self):
        """(free, total) device memory in bytes."""
        f, t = C.c_uint64(), C.c_uint64()
        _check(lib().pm_ctx_mem_info(self.h, C.byref(f), C.byref(t)))
        return f.value, t.value

    def timing(self, on):
        """0 off, 1 (True) preprocessing and leaf kernels, 2 also the step kernels."""
        _check(lib().pm_timing_enable(self.h, int(on)))

    def timing_reset(self):
        _check(lib().pm_timing_reset(self.h))

    def timing_timeline(self, path: str):
        """Append this context's timed launches (start/end on the process's time axis) to `path`."""
        _check(lib().pm_timing_timeline(self.h, str(path).encode()))

    def timing_get(self, kernel: str):
        n = C.c_uint64()
        ms = C.c_double()
        by = C.c_double()
        _check(lib().pm_timing_get(self.h, kernel.encode(), C.byref(n), C.byref(ms), C.byref(by)))
        return n.value, ms.value, by.value


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# ---------------------------------------------------------------------------
# leaf batches
# ---------------------------------------------------------------------------
def expand_key(key: bytes) -> np.ndarray:
    rk = np.zeros(44, dtype=np.uint32)
    kb = (C.c_uint8 * 16).from_buffer_copy(bytes(key))
    _check(lib().pm_expand_key(kb, _p(rk, u32p)))
    return rk


def prf_batch(rk: np.ndarray, tags, xs, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context()
    rk = np.ascontiguousarray(rk, dtype=np.uint32)
    t, x = _u64(tags), _u64(xs)
    out = np.zeros(len(t), dtype=np.uint64)
    _check(lib().pm_prf_batch(ctx.h, _p(rk, u32p), _p(t, u64p), _p(x, u64p), len(t), _p(out, u64p)))
    return out


def set_option(name: str, value: int) -> None:
    """pm_set_option: choose among equivalent kernel paths process-wide
    ("match_part", "match_part8", "match_resolve"); -2 restores the default."""
    _check(lib().pm_set_option(name.encode(), int(value)))


def l2_batch(query, rows, ctx: Context | None = None) -> np.ndarray:
    ctx = ctx or default_context()
    q = np.ascontiguousarray(query, dtype=np.float32)
    r = np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, q.shape[0])
    out = np.zeros(r.shape[0], dtype=np.float32)
    _check(lib().pm_l2_batch(ctx.h, _p(q, f32p), _p(r, f32p), r.shape[0], q.shape[0], _p(out, f32p)))
    return out


def ip_batch(query, rows, per_row: bool = True, ctx: Context | None = None):
    ctx = ctx or default_context()
    q = np.ascontiguousarray(query, dtype=np.uint32)
    r = np.ascontiguousarray(rows, dtype=np.uint32).reshape(-1, q.shape[0])
    pr = np.zeros(max(1, r.shape[0]), dtype=np.uint32)
    s = C.c_uint32()
    _check(lib().pm_ip_batch(ctx.h, _p(q, u32p), _p(r, u32p), r.shape[0], q.shape[0],
                             _p(pr, u32p) if per_row else None, C.byref(s)))
    return (pr[: r.shape[0]] if per_row else None), s.value


def ip_bench(N: int, D: int, ctx: Context | None = None, r0: int = 0, rows: int | None = None):
    """TestInnerProduct's scan fully on device; returns (sum, scan_ms).  With
    r0 / rows: only rows [r0, r0 + rows) of the N-row fill (one GPU's shard;
    the shards' sums add up mod 2^32 to the whole scan's)."""
    ctx = ctx or default_context()
    s = C.c_uint32()
    ms = C.c_double()
    if rows is None and r0 == 0:
        _check(lib().pm_ip_bench(ctx.h, N, D, C.byref(s), C.byref(ms)))
    else:
        _check(lib().pm_ip_bench_shard(ctx.h, N, D, r0, N - r0 if rows is None else rows, C.byref(s), C.byref(ms)))
    return s.value, ms.value


# ---------------------------------------------------------------------------
# PianoPIR / SimpleBatchPianoPIR
# ---------------------------------------------------------------------------
def _export(fn, h, cfg: PirConfig, *pre):
    E, PH, SS, Q = cfg.DBEntrySize, cfg.PrimaryHintNum, cfg.SetSize, cfg.MaxQueryPerChunk
    nb = SS * Q
    st = {
        "round_keys": np.zeros(44, np.uint32),
        "primary_tag": np.zeros(PH, np.uint64), "primary_parity": np.zeros(PH * E, np.uint64),
        "primary_pp": np.zeros(PH, np.uint64), "backup_tag": np.zeros(nb, np.uint64),
        "backup_parity": np.zeros(nb * E, np.uint64), "repl_idx": np.zeros(nb, np.uint64),
        "repl_val": np.zeros(nb * E, np.uint64), "hist": np.zeros(SS, np.uint64),
    }
    _check(fn(h, *pre, _p(st["round_keys"], u32p), *[_p(st[k], u64p) for k in (
        "primary_tag", "primary_parity", "primary_pp", "backup_tag", "backup_parity",
        "repl_idx", "repl_val", "hist")]))
    return st


class PianoPIR:
    """pianopir.PianoPIR (pir.go:473-548) on the GPU."""

    def __init__(self, DBSize: int, DBEntryByteNum: int, rawDB, FailureProbLog2: int,
                 seed: int = 1, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        db = _u64(rawDB)
        if db.size != DBSize * (DBEntryByteNum // 8):   # pir.go:483-485 log.Fatalf
            raise ValueError(f"Piano PIR len(rawDB) = {db.size}; want {DBSize * (DBEntryByteNum // 8)}")
        h = vp()
        _check(lib().pm_pir_create(self.ctx.h, DBSize, DBEntryByteNum, _p(db, u64p), FailureProbLog2,
                                   seed, C.byref(h)))
        self.h = h
        self.E = DBEntryByteNum // 8

    def __del__(self):
        if getattr(self, "h", None):
            lib().pm_pir_destroy(self.h)
            self.h = None

    def Preprocessing(self):
        _check(lib().pm_pir_preprocessing(self.h))

    def DummyPreprocessing(self):
        _check(lib().pm_pir_dummy_preprocessing(self.h))

    def Query(self, idx: int, realQuery: bool = True):
        """Returns (entry, err) like the Go method; err is None or QueryError."""
        out = np.zeros(self.E, dtype=np.uint64)
        st = C.c_int()
        _check(lib().pm_pir_query(self.h, idx, int(realQuery), _p(out, u64p), C.byref(st)))
        return out, (None if st.value == Q_OK else QueryError(st.value))

    def Config(self) -> dict:
        c = PirConfig()
        _check(lib().pm_pir_config_get(self.h, C.byref(c)))
        return c.asdict()

    def LocalStorageSize(self) -> float:
        return lib().pm_pir_local_storage(self.h)

    def CommCostPerQuery(self) -> float:
        return lib().pm_pir_comm_per_query(self.h)

    def PrivateQuery(self, offsets) -> np.ndarray:
        """Server answer(s) for one ([SetSize]) or many ([nq, SetSize]) offset sets."""
        o = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint32))
        ss = self.Config()["SetSize"]
        o2 = o.reshape(-1, ss)
        out = np.zeros((o2.shape[0], self.E), dtype=np.uint64)
        _check(lib().pm_pir_server_answer(self.h, _p(o2, u32p), o2.shape[0], _p(out, u64p)))
        return out[0] if o.ndim == 1 else out

    def export_state(self) -> dict:
        c = PirConfig()
        _check(lib().pm_pir_config_get(self.h, C.byref(c)))
        return _export(lib().pm_pir_export, self.h, c)


_M64 = (1 << 64) - 1


def _sm64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer of (x + golden), vectorised (pm_internal.h sm64)."""
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def synth_rows(db_seed: int, ids, E: int) -> np.ndarray:
    """Rows of the device-generated DB (pm_batchpir_create_synth): word w of
    row r = sm64(sm64(db_seed + 9) ^ (r * E + w)).  Returns len(ids) x E u64."""
    k = _sm64(np.array([(db_seed + 9) & _M64], dtype=np.uint64))[0]
    ids = np.asarray(ids, dtype=np.uint64).reshape(-1, 1)
    with np.errstate(over="ignore"):
        x = ids * np.uint64(E) + np.arange(E, dtype=np.uint64)[None, :]
    return _sm64(k ^ x)


class SimpleBatchPianoPIR:
    """pianopir.SimpleBatchPianoPIR (batch-pir.go:40-276) on the GPU."""

    def __init__(self, DBSize: int, DBEntryByteNum: int, BatchSize: int, rawDB,
                 FailureProbLog2: int, seed: int = 1, ctx: Context | None = None, _handle=None,
                 shard: int = 0, nshards: int = 1, db_seed: int | None = None):
        """shard / nshards: hold only partitions p % nshards == shard
        (pm_batchpir_create_shard); see ShardedBatchPIR for the combine.
        db_seed (with rawDB None): the DB is generated on the device,
        row r = synth_rows(db_seed, [r], E) (pm_batchpir_create_synth)."""
        self.ctx = ctx or default_context()
        self.E = DBEntryByteNum // 8
        self.shard, self.nshards = shard, nshards
        self._owned = _handle is None
        if _handle is not None:
            self.h = _handle
            return
        if db_seed is not None:   # device-generated rows (pm_batchpir_create_synth, synth_rows)
            if rawDB is not None:
                raise ValueError("pass rawDB or db_seed, not both")
            h = vp()
            _check(lib().pm_batchpir_create_synth(self.ctx.h, DBSize, DBEntryByteNum, BatchSize, FailureProbLog2,
                                                  seed, db_seed, shard, nshards, C.byref(h)))
            self.h = h
            return
        db = _u64(rawDB)
        if db.size != DBSize * self.E:   # batch-pir.go:57-59 log.Fatalf
            raise ValueError(f"BatchPIR: len(rawDB) = {db.size}; want {DBSize * self.E}")
        h = vp()
        _check(lib().pm_batchpir_create_shard(self.ctx.h, DBSize, DBEntryByteNum, BatchSize, _p(db, u64p),
                                              FailureProbLog2, seed, shard, nshards, C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None) and self._owned:
            lib().pm_batchpir_destroy(self.h)
        self.h = None

    def Client(self, seed: int, ctx: Context | None = None) -> "SimpleBatchPianoPIR":
        """Another client of this server (pm_batchpir_create_client): own keys
        (seed), hint state and counters; reads this handle's device DB in place."""
        c = SimpleBatchPianoPIR.__new__(SimpleBatchPianoPIR)
        c.ctx = ctx or self.ctx
        c.E, c.shard, c.nshards, c._owned = self.E, self.shard, self.nshards, True
        c._server = self
        h = vp()
        _check(lib().pm_batchpir_create_client(c.ctx.h, self.h, seed, C.byref(h)))
        c.h = h
        return c

    def Preprocessing(self):
        _check(lib().pm_batchpir_preprocessing(self.h))

    def DummyPreprocessing(self):
        _check(lib().pm_batchpir_dummy_preprocessing(self.h))

    def Query(self, idx):
        """Returns (responses [len(idx), DBEntrySize] uint64, err=None)."""
        ids = _u64(idx).ravel()
        out = np.zeros((len(ids), self.E), dtype=np.uint64)
        _check(lib().pm_batchpir_query(self.h, _p(ids, u64p), len(ids), _p(out, u64p)))
        return out, None

    def QueryWithMask(self, idx):
        """Query plus the per-id success mask of pm_batchpir_query_ok: True where
        the entry answers a successful sub-query, False where the id was dropped
        or its sub-query failed (entry all zero)."""
        ids = _u64(idx).ravel()
        out = np.zeros((len(ids), self.E), dtype=np.uint64)
        ok = np.zeros(len(ids), dtype=np.uint8)
        _check(lib().pm_batchpir_query_ok(self.h, _p(ids, u64p), len(ids), _p(out, u64p),
                                          ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out, ok.astype(bool)

    def QueryDevice(self, idx, dev_out: int, stream: int | None = None):
        """Query with the responses left in device memory (pm_batchpir_query_dev):
        dev_out = the address of a device buffer on this handle's GPU of
        len(idx) x (DBEntrySize + 1) uint64 words (row i: id i's entry, then its
        success flag).  stream: a HIP stream handle that is made to wait for the
        rows (e.g. torch.cuda.current_stream().cuda_stream); None: the rows are
        written when the call returns."""
        ids = _u64(idx).ravel()
        _check(lib().pm_batchpir_query_dev(self.h, _p(ids, u64p), len(ids), vp(dev_out),
                                           vp(stream) if stream else None))

    def stats(self) -> dict:
        s = BatchStats()
        _check(lib().pm_batchpir_stats_get(self.h, C.byref(s)))
        return s.asdict()

    def Config(self) -> dict:
        s = self.stats()
        return {k: s[k] for k in ("DBEntryByteNum DBEntrySize DBSize BatchSize PartitionNum "
                                  "PartitionSize ThreadNum FailureProbLog2").split()}

    def SubConfig(self, i: int) -> dict:
        c = PirConfig()
        _check(lib().pm_batchpir_subconfig(self.h, i, C.byref(c)))
        return c.asdict()

    def LocalStorageSize(self) -> float:
        return self.stats()["LocalStorage"]

    def CommCostPerBatchOnline(self) -> int:
        return int(self.stats()["CommOnline"])

    def CommCostPerBatchOffline(self) -> int:
        return int(self.stats()["CommOffline"])

    def PreprocessingTime(self) -> float:
        return self.stats()["PreprocessingTime"]

    @property
    def FinishedBatchNum(self) -> int:
        return self.stats()["FinishedBatchNum"]

    @property
    def SupportBatchNum(self) -> int:
        return self.stats()["SupportBatchNum"]

    def export_state(self, partition: int) -> dict:
        return _export(lib().pm_batchpir_export, self.h, self._cfg(partition), partition)

    def _cfg(self, i):
        c = PirConfig()
        _check(lib().pm_batchpir_subconfig(self.h, i, C.byref(c)))
        return c


# ---------------------------------------------------------------------------
# graphann
# ---------------------------------------------------------------------------
class BatchPIRGroup:
    """Clients of one server answered together (pm_batchpir_group_*): each
    Query call is, for every client s, its SimpleBatchPianoPIR.Query of
    ids[s], with all clients' sub-queries in one shared step."""

    def __init__(self, clients):
        self.clients = list(clients)   # kept alive while the group exists
        hs = (vp * len(self.clients))(*[c.h for c in self.clients])
        h = vp()
        _check(lib().pm_batchpir_group_create(hs, len(self.clients), C.byref(h)))
        self.h = h
        self.E = self.clients[0].E

    def __del__(self):
        if getattr(self, "h", None):
            lib().pm_batchpir_group_destroy(self.h)
        self.h = None

    def Preprocessing(self):
        """Every client's SimpleBatchPianoPIR.Preprocessing as one launch set."""
        _check(lib().pm_batchpir_group_preprocessing(self.h))

    def QueryWithMask(self, ids):
        """ids [S, n] -> (entries [S, n, DBEntrySize] uint64, ok [S, n] bool)."""
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        S, n = ids.shape
        if S != len(self.clients):
            raise ValueError("one row of ids per client")
        out = np.zeros((S, n, self.E), dtype=np.uint64)
        ok = np.zeros((S, n), dtype=np.uint8)
        _check(lib().pm_batchpir_group_query(self.h, _p(ids, u64p), n, _p(out, u64p),
                                             ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return out, ok.astype(bool)


class PIRGraphInfo:
    """PIRGraphInfo (private-search.go:336-531) wrapped in GraphANNFrontend
    (graphann/search.go:69-245).  nonprivate=True gives BasicGraphInfo-style
    direct vertex access."""

    def __init__(self, vectors, graph, nonprivate: bool = False, skip_prep: bool = False,
                 pir_seed: int = 1, search_seed: int = 1, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        g = np.ascontiguousarray(graph, dtype=np.uint32)
        self.N, self.Dim = v.shape
        self.M = g.shape[1]
        h = vp()
        _check(lib().pm_graph_create(self.ctx.h, self.N, self.Dim, self.M, _p(v, f32p), _p(g, u32p),
                                     int(nonprivate), int(skip_prep), pir_seed, search_seed,
                                     C.byref(h)))
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().pm_graph_destroy(self.h)
            self.h = None

    def GetMetadata(self):
        n, d, m = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().pm_graph_get_metadata(self.h, C.byref(n), C.byref(d), C.byref(m)))
        return n.value, d.value, m.value

    def GetVertexInfo(self, ids, query=None):
        """PIRGraphInfo.GetVertexInfo (private-search.go:441-506) of a batch of
        vertex ids (pm_graph_get_vertex_info): (vectors [n, dim] f32,
        neighbours [n, m] u32, ok [n] bool), plus, given a query, the L2
        distances [n] computed on the GPU beside the decode."""
        i = _u64(ids).ravel()
        n = len(i)
        vec = np.zeros((n, self.Dim), dtype=np.float32)
        nb = np.zeros((n, self.M), dtype=np.uint32)
        ok = np.zeros(n, dtype=np.uint8)
        q = None if query is None else np.ascontiguousarray(query, dtype=np.float32).ravel()
        d = np.zeros(n, dtype=np.float32) if q is not None else None
        _check(lib().pm_graph_get_vertex_info(self.h, _p(i, u64p), n, _p(vec, f32p), _p(nb, u32p), _p(ok, u8p),
                                              None if q is None else _p(q, f32p), None if d is None else _p(d, f32p)))
        return (vec, nb, ok.astype(bool)) if d is None else (vec, nb, ok.astype(bool), d)

    def GetStartVertex(self):
        """PIRGraphInfo.GetStartVertex (private-search.go:508-531): the start
        set chosen by Preprocess, (ids [k] int64, vectors [k, dim], neighbours [k, m])."""
        cnt = C.c_uint64()
        _check(lib().pm_graph_get_start_vertex(self.h, 0, None, None, None, C.byref(cnt)))
        k = cnt.value
        ids = np.zeros(k, dtype=np.uint64)
        vec = np.zeros((k, self.Dim), dtype=np.float32)
        nb = np.zeros((k, self.M), dtype=np.uint32)
        _check(lib().pm_graph_get_start_vertex(self.h, k, _p(ids, u64p), _p(vec, f32p), _p(nb, u32p), C.byref(cnt)))
        return ids.astype(np.int64), vec, nb

    def Preprocess(self):
        _check(lib().pm_graph_preprocess(self.h))

    @property
    def PIR(self) -> SimpleBatchPianoPIR | None:
        hp = lib().pm_graph_pir(self.h)
        if not hp:
            return None
        return SimpleBatchPianoPIR(0, self.Dim * 4 + self.M * 4, 0, None, 0, ctx=self.ctx,
                                   _handle=vp(hp))

    def counts(self):
        t, s = C.c_uint64(), C.c_uint64()
        _check(lib().pm_graph_counts(self.h, C.byref(t), C.byref(s)))
        return t.value, s.value

    def SearchKNN(self, query, k: int, maxStep: int, parallel: int, benchmarking: bool = False):
        q = np.ascontiguousarray(query, dtype=np.float32)
        ids = np.zeros(k, dtype=np.int64)
        steps = np.zeros(k, dtype=np.int64)
        _check(lib().pm_search_knn(self.h, _p(q, f32p), k, maxStep, parallel, int(benchmarking),
                                   _p(ids, i64p), _p(steps, i64p)))
        return ids, steps

    def SearchLoop(self, queries, k: int, step: int, parallel: int, benchmarking: bool = False):
        """private-search.go:216-240: returns (answers [q,k], online_s, maintenance_s)."""
        qs = np.ascontiguousarray(queries, dtype=np.float32)
        ans = np.zeros((qs.shape[0], k), dtype=np.int64)
        on, mt = C.c_double(), C.c_double()
        _check(lib().pm_search_loop(self.h, _p(qs, f32p), qs.shape[0], k, step, parallel,
                                    int(benchmarking), _p(ans, i64p), C.byref(on), C.byref(mt)))
        return ans, on.value, mt.value


    @classmethod
    def Shard(cls, vectors, graph, shard: int, nshards: int, pir_seed: int = 1, search_seed: int = 1,
              ctx: Context | None = None) -> "PIRGraphInfo":
        """PIRGraphInfo over shard `shard` of `nshards` of the graph DB
        (pm_graph_create_shard): this handle holds and serves the batch-PIR
        partitions p % nshards == shard only; search with search_loop_sharded."""
        s = cls.__new__(cls)
        s.ctx = ctx or default_context()
        v = np.ascontiguousarray(vectors, dtype=np.float32)
        g = np.ascontiguousarray(graph, dtype=np.uint32)
        s.N, s.Dim = v.shape
        s.M = g.shape[1]
        s.shard, s.nshards, s.synthetic = shard, nshards, None
        h = vp()
        _check(lib().pm_graph_create_shard(s.ctx.h, s.N, s.Dim, s.M, _p(v, f32p), _p(g, u32p), shard, nshards,
                                           pir_seed, search_seed, C.byref(h)))
        s.h = h
        return s

    @classmethod
    def Synthetic(cls, n: int, dim: int, m: int, data_seed: int, shard: int = 0, nshards: int = 1,
                  pir_seed: int = 1, search_seed: int = 1, ctx: Context | None = None) -> "PIRGraphInfo":
        """PIRGraphInfo over the synthetic graph of the reference's
        `-input synthetic` mode (uniform [0,1) vectors, uniform neighbours)
        generated on the device from data_seed (pm_graph_create_synth); rows
        are graph_synth_rows(n, dim, m, data_seed, ids)."""
        s = cls.__new__(cls)
        s.ctx = ctx or default_context()
        s.N, s.Dim, s.M = n, dim, m
        s.shard, s.nshards, s.synthetic = shard, nshards, data_seed
        h = vp()
        _check(lib().pm_graph_create_synth(s.ctx.h, n, dim, m, data_seed, shard, nshards, pir_seed, search_seed,
                                           C.byref(h)))
        s.h = h
        return s

    def Session(self, pir_seed: int, search_seed: int, ctx: Context | None = None) -> "PIRGraphInfo":
        """Another client session over this (preprocessed) graph and its server
        DB (pm_graph_create_session): own context, keys, hint state, start set
        and id stream; call Preprocess() on it before searching."""
        s = PIRGraphInfo.__new__(PIRGraphInfo)
        s.ctx = ctx or Context(self.ctx.device)
        s.N, s.Dim, s.M = self.N, self.Dim, self.M
        s.shard, s.nshards = getattr(self, "shard", 0), getattr(self, "nshards", 1)
        s.synthetic = getattr(self, "synthetic", None)
        s._base = self   # the base keeps the shared server alive until the session's preprocessing
        h = vp()
        _check(lib().pm_graph_create_session(s.ctx.h, self.h, pir_seed, search_seed, C.byref(h)))
        s.h = h
        return s


def search_loop_sessions(sessions, queries, k: int, step: int, parallel: int):
    """Serve len(sessions) client sessions concurrently (pm_search_loop_sessions):
    queries [S, q, dim].  Returns (answers [S, q, k], wall_s, online_s[S], maint_s[S])."""
    S = len(sessions)
    qs = np.ascontiguousarray(queries, dtype=np.float32)
    if qs.ndim != 3 or qs.shape[0] != S or qs.shape[2] != sessions[0].Dim:
        raise ValueError("queries must be [len(sessions), q, dim]")
    q = qs.shape[1]
    ans = np.zeros((S, q, k), dtype=np.int64)
    hs = (vp * S)(*[s.h for s in sessions])
    wall = C.c_double()
    on = np.zeros(S, dtype=np.float64)
    mt = np.zeros(S, dtype=np.float64)
    _check(lib().pm_search_loop_sessions(hs, S, _p(qs, f32p), q, k, step, parallel, _p(ans, i64p), C.byref(wall),
                                         on.ctypes.data_as(C.POINTER(dbl)), mt.ctypes.data_as(C.POINTER(dbl))))
    return ans, wall.value, on, mt


def search_loop_batched(sessions, queries, k: int, step: int, parallel: int, ngroups: int = 1, nthreads: int = 0):
    """Serve len(sessions) client sessions in `ngroups` concurrent lock-step
    groups, every round of a group's sessions one shared batch-PIR step
    (pm_search_loop_batched): queries [S, q, dim].
    Returns (answers [S, q, k], wall_s, online_s[S], maint_s[S])."""
    S = len(sessions)
    qs = np.ascontiguousarray(queries, dtype=np.float32)
    if qs.ndim != 3 or qs.shape[0] != S or qs.shape[2] != sessions[0].Dim:
        raise ValueError("queries must be [len(sessions), q, dim]")
    q = qs.shape[1]
    ans = np.zeros((S, q, k), dtype=np.int64)
    hs = (vp * S)(*[s.h for s in sessions])
    wall = C.c_double()
    on = np.zeros(S, dtype=np.float64)
    mt = np.zeros(S, dtype=np.float64)
    _check(lib().pm_search_loop_batched(hs, S, _p(qs, f32p), q, k, step, parallel, ngroups, nthreads, _p(ans, i64p),
                                        C.byref(wall), on.ctypes.data_as(C.POINTER(dbl)),
                                        mt.ctypes.data_as(C.POINTER(dbl))))
    return ans, wall.value, on, mt


def team_sizes(S: int, ngroups: int) -> list[int]:
    """Sessions per lock-step team, as the serving loops split them."""
    NG = max(1, min(ngroups or 1, S))
    return [S * (g + 1) // NG - S * g // NG for g in range(NG)]


def search_loop_sharded(sessions, queries, k: int, step: int, parallel: int, ngroups: int = 1, nthreads: int = 0,
                        combiner=None, model_peers: bool = False):
    """The batched serving loop over a sharded graph DB (pm_search_loop_sharded):
    every rank calls it with its own shard's sessions and the same queries
    [S, q, dim]; each shared step's per-id records are summed over the ranks by
    `combiner` (pacmann_amd.shard.RecordCombiner: an in-place all-reduce over a
    torch.distributed group), or, with model_peers (synthetic graphs), the
    other shards' answers come from the graph's spec.  Returns (answers
    [S, q, k], wall_s, online_s[S], maint_s[S])."""
    S = len(sessions)
    qs = np.ascontiguousarray(queries, dtype=np.float32)
    if qs.ndim != 3 or qs.shape[0] != S or qs.shape[2] != sessions[0].Dim:
        raise ValueError("queries must be [len(sessions), q, dim]")
    q = qs.shape[1]
    ans = np.zeros((S, q, k), dtype=np.int64)
    hs = (vp * S)(*[s.h for s in sessions])
    wall = C.c_double()
    on = np.zeros(S, dtype=np.float64)
    mt = np.zeros(S, dtype=np.float64)
    fn, bufs, user = COMBINE_FN(), None, None
    if combiner is not None:
        words = [int(lib().pm_sharded_record_words(sessions[0].h, n, parallel)) for n in team_sizes(S, ngroups)]
        if getattr(combiner, "native", False):   # pm_rccl_combine: the C entry point itself, no Python per step
            user = combiner.prepare(words)
            fn = COMBINE_FN(C.cast(lib().pm_rccl_combine, vp).value)
        else:
            ptrs = combiner.prepare(words)
            bufs = (vp * len(ptrs))(*ptrs)
            fn = COMBINE_FN(combiner.callback)
    rc = lib().pm_search_loop_sharded(hs, S, _p(qs, f32p), q, k, step, parallel, ngroups, nthreads, fn, user, bufs,
                                      int(model_peers), _p(ans, i64p), C.byref(wall),
                                      on.ctypes.data_as(C.POINTER(dbl)), mt.ctypes.data_as(C.POINTER(dbl)))
    if combiner is not None:
        combiner.finish()   # raises the combine's own exception first
    _check(rc)
    return ans, wall.value, on, mt


def graph_synth_rows(n: int, dim: int, m: int, data_seed: int, ids):
    """Rows of the synthetic graph (pm_graph_synth_rows): (vectors [k, dim] f32,
    neighbours [k, m] u32) of vertices `ids`."""
    i = _u64(ids).ravel()
    vec = np.zeros((len(i), dim), dtype=np.float32)
    nb = np.zeros((len(i), m), dtype=np.uint32)
    _check(lib().pm_graph_synth_rows(n, dim, m, data_seed, _p(i, u64p), len(i), _p(vec, f32p), _p(nb, u32p)))
    return vec, nb


def knn(base, queries, k: int, ctx: Context | None = None, with_dist: bool = False):
    """Exact k nearest base rows of each query by (L2Dist, id) (pm_knn): the
    ground truth of graphann.ComputeRecall.  ids [nq, k] int64, -1 padded."""
    ctx = ctx or default_context()
    b = np.ascontiguousarray(base, dtype=np.float32)
    q = np.ascontiguousarray(queries, dtype=np.float32).reshape(-1, b.shape[1])
    ids = np.zeros((q.shape[0], k), dtype=np.int64)
    d = np.zeros((q.shape[0], k), dtype=np.float32)
    _check(lib().pm_knn(ctx.h, _p(b, f32p), b.shape[0], b.shape[1], _p(q, f32p), q.shape[0], k, _p(ids, i64p),
                        _p(d, f32p)))
    return (ids, d) if with_dist else ids


def build_graph(vectors, m: int, alpha: float = 1.2, seed: int = 1, ctx: Context | None = None):
    """graphann.BuildGraph (build_graph.go:97-105,314-523) on the GPU with exact
    kNN candidates (pm_build_graph).  Returns (graph [n, m] uint32, times dict)."""
    ctx = ctx or default_context()
    v = np.ascontiguousarray(vectors, dtype=np.float32)
    g = np.zeros((v.shape[0], m), dtype=np.uint32)
    t = (dbl * 4)()
    _check(lib().pm_build_graph(ctx.h, _p(v, f32p), v.shape[0], v.shape[1], m, alpha, seed, _p(g, u32p), t))
    return g, {"knn_s": t[0], "prune1_s": t[1], "host_edges_s": t[2], "prune2_s": t[3]}


GraphANNFrontend = PIRGraphInfo
