"""Check the bench line's rooflines against rocprofv3's own kernel timings.

    python tools/prof_check.py TRACE_CSV[.gz] BENCH_JSON OUT_JSON [UNTRACED_BENCH_JSON]

TRACE_CSV is the `--kernel-trace` output of a `rocprofv3 ... -- python3
bench.py` run and BENCH_JSON the line that same run printed.  Every roofline
object in the line that names its kernel symbol and launch shape
(`symbol`, `grid_threads`, see bench.py attach_traffic) is matched with the
dispatches of that symbol and shape in the trace; the output lists, per
roofline, the bench's live average (HIP events on the launch's own stream)
beside rocprof's average over the same shape, and `frac` recomputed from
rocprof's time (algorithmic bytes per launch / rocprof average / peak).
Launch shapes are total work-items (Grid_Size_X * Y * Z).
"""
import csv
import gzip
import json
import sys
from collections import defaultdict


def load_trace(path):
    op = gzip.open if path.endswith(".gz") else open
    by = defaultdict(list)
    with op(path, "rt") as fh:
        for r in csv.DictReader(fh):
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            by[(r["Kernel_Name"], g)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for k in by:
        by[k].sort()
    return by


def timed_window(spans, n, gap_ns=50e6):
    """The bench's timed launches among a shape's dispatches: the dispatches are
    cut into runs at idle gaps > 50 ms (warm-up + timed region, then e.g. the
    isolated one-group run); the timed region is the last n of the first run
    holding at least n.  None if no run does."""
    runs, cur = [], [spans[0]]
    for a in spans[1:]:
        if a[0] - cur[-1][1] > gap_ns:
            runs.append(cur)
            cur = [a]
        else:
            cur.append(a)
    runs.append(cur)
    for r in runs:
        if len(r) >= n:
            return r[-n:]
    return None


def rooflines(obj, path=""):
    """(json path, dict) of every roofline-like object carrying symbol + grid."""
    if isinstance(obj, dict):
        if "symbol" in obj and "grid_threads" in obj and obj.get("avg_ms"):
            yield path, obj
        for k, v in obj.items():
            yield from rooflines(v, f"{path}.{k}" if path else k)


def lookup(obj, path):
    for k in path.split("."):
        obj = obj.get(k) if isinstance(obj, dict) else None
    return obj


def main():
    trace, bench, out = sys.argv[1:4]
    # optional: the line of the same command run WITHOUT the profiler (the
    # driver's kind of run); under rocprofv3's kernel trace the HIP events of
    # kernels that share the GPU with other streams' kernels read longer than
    # the trace's own timestamps, while the untraced line's events agree with them
    plain = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else None
    by = load_trace(trace)
    line = json.load(open(bench))
    rows = []
    for path, r in rooflines(line):
        spans = by.get((r["symbol"], int(r["grid_threads"])), [])
        ms = [(b - a) / 1e6 for a, b in spans]
        row = {"roofline": path, "kernel": r.get("kernel"), "grid_threads": r["grid_threads"],
               "bench_avg_ms": r["avg_ms"], "bench_frac": r.get("frac"),
               "rocprof_dispatches": len(ms)}
        if ms:
            avg = sum(ms) / len(ms)
            row["rocprof_avg_ms"] = round(avg, 5)
            row["ratio_bench_over_rocprof"] = round(r["avg_ms"] / avg, 4)
            if r.get("alg_bytes_per_launch") and r.get("peak"):
                row["frac_from_rocprof"] = round(r["alg_bytes_per_launch"] / (avg / 1e3) / 1e9 / r["peak"], 4)
            # the same over the bench's own timed launches only (its `launches` count)
            n = int(r.get("launches") or 0)
            win = timed_window(spans, n) if 0 < n < len(spans) else None
            if win:
                tavg = sum((b - a) / 1e6 for a, b in win) / n
                row["rocprof_timed_dispatches"] = n
                row["rocprof_timed_avg_ms"] = round(tavg, 5)
                row["ratio_bench_over_rocprof_timed"] = round(r["avg_ms"] / tavg, 4)
        u = lookup(plain, path) if plain else None
        if u and u.get("avg_ms") and "rocprof_avg_ms" in row:
            ref = row.get("rocprof_timed_avg_ms", row["rocprof_avg_ms"])
            row["untraced_bench_avg_ms"] = u["avg_ms"]
            row["ratio_untraced_bench_over_rocprof"] = round(u["avg_ms"] / ref, 4)
        rows.append(row)
    json.dump({"trace": trace, "bench_line": bench, "untraced_line": sys.argv[4] if plain else None,
               "rooflines": rows}, open(out, "w"), indent=1)
    for row in rows:
        print(f"{row['roofline']:<45} bench {row['bench_avg_ms']:.5f} ms  rocprof "
              f"{row.get('rocprof_avg_ms', float('nan')):.5f} ms ({row['rocprof_dispatches']} dispatches)  "
              f"ratio {row.get('ratio_bench_over_rocprof', float('nan'))}"
              + (f"; timed launches {row['rocprof_timed_avg_ms']:.5f} ms ratio {row['ratio_bench_over_rocprof_timed']}"
                 if "rocprof_timed_avg_ms" in row else "")
              + (f"; untraced line {row['untraced_bench_avg_ms']:.5f} ms ratio {row['ratio_untraced_bench_over_rocprof']}"
                 if "untraced_bench_avg_ms" in row else ""))


if __name__ == "__main__":
    main()
