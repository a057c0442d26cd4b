"""Summarise two rocprofv3 counter passes (FETCH_SIZE and WRITE_SIZE, collected
in separate `--pmc` runs of the same command) into per-kernel HBM bytes per
dispatch, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE
reports half the bytes of 16-B-per-lane loads, so it is doubled; WRITE_SIZE is
taken as is.  Both counters are in KB.

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv OUT.json "command run"
"""
import csv
import gzip
import json
import sys
from collections import defaultdict


def per_kernel(path, counter, by_grid=False):
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(gzip.open(path, 'rt') if path.endswith('.gz') else open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = acc[(r["Kernel_Name"], int(r["Grid_Size"])) if by_grid else r["Kernel_Name"]]
        k[0] += 1
        k[1] += float(r["Counter_Value"])
    return {name: (n, tot / n) for name, (n, tot) in acc.items()}


def main():
    fetch_csv, write_csv, out, cmd = sys.argv[1:5]
    fetch = per_kernel(fetch_csv, "FETCH_SIZE")
    write = per_kernel(write_csv, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fetch) | set(write)):
        k = {}
        if name in fetch:
            k["dispatches"] = fetch[name][0]
            k["FETCH_SIZE_KB_avg"] = fetch[name][1]
        if name in write:
            k["WRITE_SIZE_KB_avg"] = write[name][1]
        if name in fetch and name in write:
            k["hbm_bytes_per_dispatch_corrected"] = fetch[name][1] * 2 * 1024 + write[name][1] * 1024
        kernels[name] = k
    # the same per launch shape (Grid_Size, threads): one kernel serves several
    # workloads of the bench (e.g. the BIGANN-100M and -1B folds)
    fg, wg = per_kernel(fetch_csv, "FETCH_SIZE", True), per_kernel(write_csv, "WRITE_SIZE", True)
    for (name, grid) in sorted(set(fg) & set(wg)):
        kernels[name].setdefault("by_grid", {})[str(grid)] = {
            "dispatches": fg[(name, grid)][0],
            "hbm_bytes_per_dispatch_corrected": fg[(name, grid)][1] * 2 * 1024 + wg[(name, grid)][1] * 1024}
    json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, two separate passes of `{cmd}` "
                         "on one MI355X; units KB per dispatch; gfx950 correction per MI355X_MICROARCH.md "
                         "§HBM: FETCH_SIZE x2 for 16-B/lane loads",
               "kernels": kernels}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
