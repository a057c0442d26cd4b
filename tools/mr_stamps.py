"""Phase breakdown of k_match_resolve_s from a PM_MR_STAMPS build's stamp file.

    python tools/mr_stamps.py STAMPS.bin

Per recorded step: the kernel's span (first workgroup start to last end,
s_memrealtime at 100 MHz), the mean per-workgroup time of each phase (0 start
-> 1 partition record -> 2 match loads + ballots -> 3 all waves' matches ->
4 candidates' tags -> 5 chain + flush -> 6 expansion guesses -> 7 query sets
issued) and the mean workgroup lifetime.
"""
import sys

import numpy as np

NAMES = ["part", "match", "barrier", "tags", "chain", "guess", "qset"]


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    off, rows = 0, []
    while off < raw.size:
        n = int(raw[off])
        t = raw[off + 1: off + 1 + n * 8].reshape(n, 8).astype(np.int64)
        off += 1 + n * 8
        t = t[(t[:, 0] > 0) & (t[:, 7] > 0)]
        if not len(t):
            continue
        for i in range(1, 8):   # a phase a workgroup skipped: its previous stamp
            t[:, i] = np.where(t[:, i] == 0, t[:, i - 1], t[:, i])
        span = (t[:, 7].max() - t[:, 0].min()) / 100
        life = (t[:, 7] - t[:, 0]) / 100
        rows.append([len(t), span, life.mean()] + [(t[:, i + 1] - t[:, i]).mean() / 100 for i in range(7)])
    a = np.array(rows)
    print(f"{len(a)} steps, {a[:, 0].mean():.0f} workgroups each")
    print(f"kernel span {a[:, 1].mean():.2f} us (min {a[:, 1].min():.2f}), workgroup lifetime {a[:, 2].mean():.2f} us")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:<8} {a[:, 3 + i].mean():7.2f} us")


if __name__ == "__main__":
    main()
