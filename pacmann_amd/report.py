"""Harness side of the private search.

Restates, on top of the GPU path, what `private-search.go:main` does around
the query loop: the recall evaluation (`graphann/build_graph.go:821-863`,
`ComputeRecall`), the int-matrix files of answers / ground truth
(`graphann/loader.go:217-364`), and the report block (`private-search.go:
286-331`) with the same fields, formulas and formatting, so a report written
here reads like `private-search-report.txt`.

Pure host code: nothing here computes on the device.
"""
from __future__ import annotations

import os
import time

import numpy as np


def compute_recall(gnd, response, k: int) -> float:
    """ComputeRecall (build_graph.go:821-863): recall@k with the top-k ground
    truth as the relevant set; a repeated answer within a row is skipped.
    float32 accumulation as in the reference."""
    response = [list(map(int, r)) for r in response]
    gnd = [list(map(int, g)) for g in gnd]
    nq = len(response)
    recall = np.float32(0.0)
    for i in range(nq):
        row, truth = response[i], gnd[i]
        hit = 0
        for j in range(k):
            if row[j] in row[:j]:
                continue
            if row[j] in truth[:k]:
                hit += 1
        recall = np.float32(recall + np.float32(hit) / np.float32(k))
    return float(np.float32(recall / np.float32(nq)))


def save_int_matrix(path: str, matrix) -> None:
    """SaveIntMatrixToFile (loader.go:306-364): .npy as int32 [n, m], .txt as
    space-terminated rows."""
    m = np.asarray(matrix)
    ext = os.path.splitext(path)[1]
    if ext == ".npy":
        np.save(path, m.astype(np.int32))
    elif ext == ".txt":
        with open(path, "w") as f:
            for row in m:
                f.write("".join(f"{int(x)} " for x in row) + "\n")
    else:
        raise ValueError(f"unknown file extension: {ext}")


def load_int_matrix(path: str, n: int, m: int) -> np.ndarray:
    """LoadIntMatrixFromFile (loader.go:91-116, 217-304): .npy (int32, at least
    n rows of m), .txt (m fields per line), .ivecs (uint32 rows with a 4-byte
    dimension prefix)."""
    ext = os.path.splitext(path)[1]
    if ext == ".npy":
        a = np.load(path, allow_pickle=False)
        if a.ndim != 2 or a.shape[0] < n or a.shape[1] != m:
            raise ValueError(f"invalid shape: {list(a.shape)}")
        return a[:n].astype(np.int64)
    if ext == ".txt":
        rows = []
        with open(path) as f:
            for i, line in zip(range(n), f):
                fields = line.split()
                if len(fields) != m:
                    raise ValueError(f"line {i + 1} has {len(fields)} fields, expected {m}")
                rows.append([int(x) for x in fields])
        out = np.zeros((n, m), dtype=np.int64)
        if rows:
            out[:len(rows)] = rows
        return out
    if ext == ".ivecs":
        raw = np.fromfile(path, dtype=np.uint32)
        out, pos = [], 0
        for _ in range(n):
            d = int(raw[pos])
            out.append(raw[pos + 1:pos + 1 + d].astype(np.int64))
            pos += 1 + d
        return np.stack(out)
    raise ValueError(f"unknown file extension: {ext}")


def format_report(*, n: int, db_bytes: int, k: int, step: int, parallel: int, rtt_ms: int, seed: int,
                  window: int, storage: float, prep_time: float, offline_comm: float,
                  support_batch_num: int, avg_time: float, online_comm: float, recall: float) -> str:
    """The report block of private-search.go:293-330, byte for byte."""
    main_per_q = prep_time / float(support_batch_num) * float(step) * float(parallel)
    lines = [
        "-------------------------",
        "Private ANN Benchmarking w/ Go Frontend",
        "Settings:",
        f"** Vector Num: {n}",
        f"** DB Size (MB): {db_bytes / 1024.0 / 1024.0:f}",
        f"** Top K: {k}",
        f"** Rounds: {step}",
        f"** Parallel Exploration: {parallel}",
        f"** RTT (ms): {rtt_ms}",
        f"** Random Seed: {seed}",
        f"** Window Size: {window}",
        "",
        "Preprocessing Cost:",
        f"** Storage (MB): {storage / 1024.0 / 1024.0:f}",
        f"** Preparation Time (s): {prep_time:f}",
        f"** Offline Communication Cost Per Q (KB, amt.): {offline_comm * step * parallel / 1024.0:f}",
        f"** Amortized Maintainence Time Per Q (s): {main_per_q:f}",
        "",
        "Online Cost:",
        f"** Average Computation Time Per Query (s): {avg_time:f}",
        f"** Average Total Time Per Q (s): {avg_time + rtt_ms / 1000.0 * step:f}",
        f"** Online Communication Per Q (KB): {online_comm * step * parallel / 1024.0:f}",
        "",
        "Quality:",
        f"** Recall: {recall:f}",
        "-----------------------",
    ]
    return "\n".join(lines) + "\n"


def report_fields(pir_stats: dict, *, n: int, k: int, step: int, parallel: int) -> dict:
    """The PIR-derived report inputs (private-search.go:211, 294-301)."""
    return {
        "n": n,
        "db_bytes": int(pir_stats["DBSize"]) * int(pir_stats["DBEntryByteNum"]),
        "window": int(pir_stats["SupportBatchNum"]) // (step * parallel),
        "storage": float(pir_stats["LocalStorage"]),
        "prep_time": float(pir_stats["PreprocessingTime"]),
        "offline_comm": float(pir_stats["CommOffline"]),
        "online_comm": float(pir_stats["CommOnline"]),
        "support_batch_num": int(pir_stats["SupportBatchNum"]),
        "k": k, "step": step, "parallel": parallel,
    }


def private_search(frontend, queries, *, k: int = 10, step: int = 20, parallel: int = 3, rtt_ms: int = 0,
                   seed: int = 1, gnd=None, output_file: str | None = None, report_file: str | None = None,
                   benchmarking: bool = False) -> dict:
    """private-search.go:196-331 over a preprocessed GraphANNFrontend: the
    query loop with maintenance (pm_search_loop), averages, success counts,
    answers file, recall and the appended report."""
    q = np.asarray(queries, dtype=np.float32)
    t0 = time.perf_counter()
    answers, online_s, maint_s = frontend.SearchLoop(q, k, step, parallel, benchmarking)
    wall = time.perf_counter() - t0
    nq = q.shape[0]
    total, succ = frontend.counts()
    out = {
        "answers": answers,
        "avg_time": online_s / nq,
        "avg_maintenance_time": maint_s / nq,
        "wall_s": wall,
        "total_query_num": total,
        "succ_query_num": succ,
        "success_rate": float(np.float32(succ) / np.float32(total)) if total else 0.0,
        "recall": -1.0,
    }
    if output_file:
        save_int_matrix(output_file, answers)
    if gnd is not None:
        out["recall"] = compute_recall(gnd, answers, k)
    pir = frontend.PIR
    if pir is not None:
        f = report_fields(pir.stats(), n=frontend.N, k=k, step=step, parallel=parallel)
        out["report"] = format_report(rtt_ms=rtt_ms, seed=seed, avg_time=out["avg_time"],
                                      recall=out["recall"], **f)
        if report_file:
            with open(report_file, "a") as fh:
                fh.write(out["report"])
    return out


# ---------------------------------------------------------------------------
# MS-MARCO end-to-end quality (behaviour of reproduction/msmarco/evaluate.py):
# the search returns vector ids; a vector id names a passage through the
# corpus's docid list; a query scores 1/rank of the first returned passage that
# is its relevant one.  Written from that behaviour, not from the script.
# ---------------------------------------------------------------------------
def _lines(path):
    with open(path, encoding="utf-8") as fh:
        yield from enumerate(fh, start=1)


def read_queries_tsv(path: str) -> list[tuple[str, str]]:
    """(qid, text) pairs of a tab-separated query file, kept in file order.
    The text is everything after the first tab."""
    pairs = []
    for ln, raw in _lines(path):
        qid, tab, text = raw.rstrip("\r\n").partition("\t")
        if not tab:
            raise ValueError(f"{path}:{ln}: expected 'qid<TAB>text'")
        pairs.append((qid, text))
    return pairs


def read_qrels(path: str) -> dict[str, str]:
    """Relevance judgements in TREC form (`qid iter docid rel`).  A query keeps
    the docid of its earliest line; later lines for it are ignored."""
    first: dict[str, str] = {}
    for ln, raw in _lines(path):
        cols = raw.split()
        if len(cols) != 4:
            raise ValueError(f"{path}:{ln}: expected 4 columns, got {len(cols)}")
        first.setdefault(cols[0], cols[2])
    return first


def read_results(path: str, query_count: int, k: int) -> np.ndarray:
    """The search output as a (query_count, k) int64 matrix, from either an
    integer .npy array (detected by its magic bytes) or whitespace-separated
    text with one query per line."""
    with open(path, "rb") as fh:
        is_npy = fh.read(6) == b"\x93NUMPY"
    if is_npy:
        arr = np.load(path, allow_pickle=False)
        if arr.dtype.kind not in "iu":
            raise ValueError(f"{path}: integer ids expected, array dtype is {arr.dtype}")
    else:
        table = [[int(tok) for tok in raw.split()] for _, raw in _lines(path)]
        widths = {len(r) for r in table}
        if widths - {k}:
            bad = next(i for i, r in enumerate(table, start=1) if len(r) != k)
            raise ValueError(f"{path}:{bad}: {len(table[bad - 1])} ids on the line, k is {k}")
        arr = np.asarray(table, dtype=np.int64).reshape(len(table), k)
    if arr.shape != (query_count, k):
        raise ValueError(f"{path}: results are {arr.shape}, need {(query_count, k)}")
    return arr.astype(np.int64)


def mrr_at_k(results, queries: list[tuple[str, str]], qrels: dict[str, str], docids,
             output_docids: str | None = None) -> dict:
    """Mean reciprocal rank of the relevant passage over every query (0 for a
    query whose passage is not returned).  A vector id outside [0, len(docids))
    maps to the placeholder "INVALID_VECTOR_ID" and matches nothing.  Every
    query must have a judgement (KeyError otherwise).  output_docids, if given,
    receives for each query a "Query: <qid> <text>" line, its returned docids
    one per line, then a "----------" line and a blank line."""
    res = np.asarray(results)
    ncorpus = len(docids)
    rr_sum, found = 0.0, 0
    listing: list[str] = []
    for row, (qid, text) in zip(res, queries):
        target = qrels[qid]
        names = [str(docids[v]) if 0 <= v < ncorpus else "INVALID_VECTOR_ID" for v in row]
        listing += [f"Query: {qid} {text}", *names, "----------", ""]
        rank = next((r for r, name in enumerate(names, start=1) if name == target), 0)
        if rank:
            found += 1
            rr_sum += 1.0 / rank
    if output_docids:
        with open(output_docids, "w", encoding="utf-8") as fh:
            fh.write("".join(s + "\n" for s in listing))
    nq = len(queries)
    width = res.shape[1] if res.ndim == 2 else 0
    return {"metric": f"MRR@{width}", "mrr": rr_sum / nq if nq else 0.0, "queries": nq, "ranked_queries": found}
