"""On-disk vector / graph formats of the reference (graphann/loader.go), host side.

SURVEY.md §8(f) rank 3: what a real SIFT / MS-MARCO run needs to feed the
engine.  Every reader returns numpy arrays in the layout the engine takes
(float32 [n, dim] vectors, int64 [n, m] graphs / id matrices); the semantics
follow loader.go case by case, including its edge behaviour:

* ``.bvecs`` (LoadBvecsFile :16-58): records ``<int32 dim><dim x uint8>``; a
  file shorter than ``n`` records leaves the remaining rows zero (the Go code
  prints "Unexpected EOF" and returns what it has); a longer record is cut to
  ``dim`` (``copy`` semantics).
* ``.fvecs`` (LoadFvecsFile :64-84): records ``<int32 dim><dim x float32>``;
  reading stops at the first short record, so fewer than ``n`` rows may come back.
* ``.ivecs`` (LoadIvecsFile :90-115): records ``<int32 dim><dim x uint32>``; a
  short file is an error (the Go code panics).
* ``.txt`` (LoadTxtFileFloat32 :121-153, LoadGraphFromTxtFile :237-269): one
  row per line, exactly ``dim`` whitespace-separated fields, else an error;
  missing lines leave zero rows.  Floats are parsed to float32 like
  ``strconv.ParseFloat(s, 32)``.
* ``.npy`` vectors (LoadFloat32MatrixFromNpy :160-188): a 2-D **float64** array
  with at least ``n`` rows and exactly ``dim`` columns, converted to float32.
* ``.npy`` graphs (LoadGraphFromNpyFile :210-235): a 2-D **int32** array, shape
  (>= n, m).
* writers (SaveGraphToNpyFile :306-326, SaveGraphToTxtFile :328-348): int32
  ``(n, m)`` npy, and ``"%d "`` per entry with a newline per row.

npy files are read with ``allow_pickle=False``.
"""
from __future__ import annotations

import os
import sys

import numpy as np

__all__ = ["load_float32_matrix", "load_bvecs", "load_fvecs", "load_ivecs", "load_txt_float32",
           "load_npy_float32", "load_graph", "load_graph_npy", "load_graph_txt", "save_graph",
           "save_graph_npy", "save_graph_txt", "load_int_matrix", "save_int_matrix_file"]


class LoaderError(ValueError):
    pass


def _ext(path: str) -> str:
    return os.path.splitext(str(path))[1]


def _map(path) -> np.ndarray:
    """The file as a read-only byte map: only the pages a reader touches are
    read, so asking for the first n records of a 132 GB bigann_base.bvecs
    reads n records, not the file (loader.go streams them the same way)."""
    if os.path.getsize(path) == 0:
        return np.zeros(0, dtype=np.uint8)
    return np.memmap(path, dtype=np.uint8, mode="r")


def _uniform_prefix(raw: np.ndarray, item: int, n: int):
    """(rows, d) when the first min(n, whole records) records all carry the
    first record's dimension d and nothing past them could be read as another
    record of the first n (so the record walk would return the same rows);
    else None.  Only those rows' prefixes are inspected."""
    if raw.size < 4:
        return None
    d = int(raw[:4].view("<i4")[0])
    if d <= 0:
        return None
    rec = 4 + d * item
    rows = min(n, raw.size // rec)
    if rows < n and raw.size - rows * rec >= 4:
        return None   # a partial tail record: let the walk decide what it holds
    dims = np.asarray(raw[:rows * rec]).reshape(rows, rec)[:, :4].copy().view("<i4").ravel()
    if not (dims == d).all():
        return None
    return rows, d


def _records(raw: np.ndarray, item: int, n: int):
    """Yield (dim, payload bytes) for at most n records; stops at a short one."""
    off = 0
    for _ in range(n):
        if off + 4 > raw.size:
            return
        d = int(raw[off:off + 4].view("<i4")[0])
        end = off + 4 + d * item
        if d < 0 or end > raw.size:
            return
        yield d, np.asarray(raw[off + 4:end])
        off = end


def _body(raw: np.ndarray, rows: int, d: int, item: int) -> np.ndarray:
    rec = 4 + d * item
    return np.asarray(raw[:rows * rec]).reshape(rows, rec)[:, 4:]


def load_bvecs(path, n: int, dim: int) -> np.ndarray:
    raw = _map(path)
    out = np.zeros((n, dim), dtype=np.float32)
    u = _uniform_prefix(raw, 1, n)
    if u is not None:
        rows, d = u
        w = min(d, dim)
        out[:rows, :w] = _body(raw, rows, d, 1)[:, :w]
        if rows < n:
            print("Unexpected EOF", file=sys.stderr)
        return out
    i = 0
    for d, payload in _records(raw, 1, n):
        w = min(d, dim)
        out[i, :w] = payload[:w]
        i += 1
    if i < n:
        print("Unexpected EOF", file=sys.stderr)
    return out


def load_fvecs(path, n: int, dim: int) -> np.ndarray:
    """Rows as stored (their own dimension); stops at the first short record."""
    raw = _map(path)
    u = _uniform_prefix(raw, 4, n)
    if u is not None:
        rows, d = u
        return _body(raw, rows, d, 4).copy().view("<f4").astype(np.float32)
    rows = [p.copy().view("<f4").astype(np.float32) for _, p in _records(raw, 4, n)]
    if not rows:
        return np.zeros((0, dim), dtype=np.float32)
    if len({r.size for r in rows}) != 1:
        raise LoaderError("ragged fvecs rows: dimensions differ")
    return np.stack(rows)


def load_ivecs(path, n: int, dim: int) -> np.ndarray:
    raw = _map(path)
    u = _uniform_prefix(raw, 4, n)
    if u is not None:
        rows, d = u
        if rows < n:
            raise LoaderError(f"Error reading vector {rows}: unexpected EOF")
        return _body(raw, rows, d, 4).copy().view("<u4").astype(np.int64)
    rows = [p.copy().view("<u4").astype(np.int64) for _, p in _records(raw, 4, n)]
    if len(rows) < n:
        raise LoaderError(f"Error reading vector {len(rows)}: unexpected EOF")
    if len({r.size for r in rows}) != 1:
        raise LoaderError("ragged ivecs rows: dimensions differ")
    return np.stack(rows)


def _txt_rows(path, n: int, dim: int, conv):
    out = []
    with open(path, "r") as f:
        for i, line in enumerate(f):
            if i == n:
                break
            fields = line.split()
            if len(fields) != dim:
                raise LoaderError(f"line {i + 1} has {len(fields)} fields, expected {dim}")
            try:
                out.append([conv(x) for x in fields])
            except ValueError as e:
                raise LoaderError(f"failed to parse a field on line {i + 1}: {e}") from None
    return out


def load_txt_float32(path, n: int, dim: int) -> np.ndarray:
    out = np.zeros((n, dim), dtype=np.float32)
    rows = _txt_rows(path, n, dim, float)
    if rows:   # float64 parse, then one rounding to float32 == ParseFloat(s, 32)
        out[:len(rows)] = np.asarray(rows, dtype=np.float64).astype(np.float32)
    return out


def load_npy_float32(path, n: int, dim: int) -> np.ndarray:
    a = np.load(path, allow_pickle=False, mmap_mode="r")
    if a.ndim != 2 or a.shape[0] < n or a.shape[1] != dim:
        raise LoaderError(f"invalid shape: {list(a.shape)}, expected ({n}, {dim})")
    if a.dtype != np.float64:
        raise LoaderError(f"npy vectors must be float64 (gonpy GetFloat64), got {a.dtype}")
    return np.ascontiguousarray(a[:n], dtype=np.float64).astype(np.float32)


def load_float32_matrix(path, n: int, dim: int) -> np.ndarray:
    """LoadFloat32Matrix (loader.go:197-215): dispatch on the extension."""
    ext = _ext(path)
    if ext == ".bvecs":
        return load_bvecs(path, n, dim)
    if ext == ".fvecs":
        return load_fvecs(path, n, dim)
    if ext == ".txt":
        return load_txt_float32(path, n, dim)
    if ext == ".npy":
        return load_npy_float32(path, n, dim)
    raise LoaderError(f"unknown file extension: {ext}")


def load_graph_npy(path, n: int, m: int) -> np.ndarray:
    a = np.load(path, allow_pickle=False, mmap_mode="r")
    if a.ndim != 2 or a.shape[0] < n or a.shape[1] != m:
        raise LoaderError(f"invalid shape: {list(a.shape)}")
    if a.dtype != np.int32:
        raise LoaderError(f"npy graphs must be int32 (gonpy GetInt32), got {a.dtype}")
    return np.asarray(a[:n], dtype=np.int64)


def load_graph_txt(path, n: int, m: int) -> np.ndarray:
    out = np.zeros((n, m), dtype=np.int64)
    rows = _txt_rows(path, n, m, int)
    if rows:
        out[:len(rows)] = np.asarray(rows, dtype=np.int64)
    return out


def load_graph(path, n: int, m: int) -> np.ndarray:
    """LoadGraphFromFile / LoadIntMatrixFromFile (loader.go:287-304)."""
    ext = _ext(path)
    if ext == ".npy":
        return load_graph_npy(path, n, m)
    if ext == ".txt":
        return load_graph_txt(path, n, m)
    if ext == ".ivecs":
        return load_ivecs(path, n, m)
    raise LoaderError(f"unknown file extension: {ext}")


load_int_matrix = load_graph


def save_graph_npy(path, graph) -> None:
    g = np.asarray(graph)
    if g.ndim != 2:
        raise LoaderError("graph must be 2-D")
    np.save(path, g.astype(np.int32), allow_pickle=False)


def save_graph_txt(path, graph) -> None:
    g = np.asarray(graph, dtype=np.int64)
    with open(path, "w") as f:
        for row in g:
            f.write("".join(f"{int(x)} " for x in row))
            f.write("\n")


def save_graph(path, graph) -> None:
    """SaveGraphToFile / SaveIntMatrixToFile (loader.go:350-364)."""
    ext = _ext(path)
    if ext == ".npy":
        return save_graph_npy(path, graph)
    if ext == ".txt":
        return save_graph_txt(path, graph)
    raise LoaderError(f"unknown file extension: {ext}")


save_int_matrix_file = save_graph
