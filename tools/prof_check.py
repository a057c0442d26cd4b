"""Check the bench line's rooflines against rocprofv3's own kernel timings.

    python tools/prof_check.py TRACE_CSV[.gz] BENCH_JSON OUT_JSON

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
            by[(r["Kernel_Name"], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return by


def rooflines(obj, path=""):
    """(json path, dict) of every roofline-like object carrying symbol + grid."""
    if isinstance(obj, dict):
        if "symbol" in obj and "grid_threads" in obj and obj.get("avg_ms"):
            yield path, obj
        for k, v in obj.items():
            yield from rooflines(v, f"{path}.{k}" if path else k)


def main():
    trace, bench, out = sys.argv[1:4]
    by = load_trace(trace)
    line = json.load(open(bench))
    rows = []
    for path, r in rooflines(line):
        ms = by.get((r["symbol"], int(r["grid_threads"])), [])
        row = {"roofline": path, "kernel": r.get("kernel"), "grid_threads": r["grid_threads"],
               "bench_avg_ms": r["avg_ms"], "bench_frac": r.get("frac"),
               "rocprof_dispatches": len(ms)}
        if ms:
            avg = sum(ms) / len(ms)
            row["rocprof_avg_ms"] = round(avg, 5)
            row["ratio_bench_over_rocprof"] = round(r["avg_ms"] / avg, 4)
            if r.get("alg_bytes_per_launch") and r.get("peak"):
                row["frac_from_rocprof"] = round(r["alg_bytes_per_launch"] / (avg / 1e3) / 1e9 / r["peak"], 4)
        rows.append(row)
    json.dump({"trace": trace, "bench_line": bench, "rooflines": rows}, open(out, "w"), indent=1)
    for row in rows:
        print(f"{row['roofline']:<45} bench {row['bench_avg_ms']:.5f} ms  rocprof "
              f"{row.get('rocprof_avg_ms', float('nan')):.5f} ms ({row['rocprof_dispatches']} dispatches)  "
              f"ratio {row.get('ratio_bench_over_rocprof', float('nan'))}")


if __name__ == "__main__":
    main()
