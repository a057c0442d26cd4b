"""Phase breakdown of k_answer from a PM_ANSWER_STAMPS build's stamp file.

    python tools/answer_stamps.py STAMPS.bin

Per recorded step: the kernel's span (first workgroup start to last
workgroup end, s_memrealtime at 100 MHz), the mean per-workgroup time in
each phase (0 start -> 1 resolution read -> 2 query set in LDS -> 3 gather
reduced -> 4 decoded -> 5 results issued), the mean workgroup lifetime, and
the mean number of workgroups in flight (sum of lifetimes / span).
"""
import sys

import numpy as np


def main():
    raw = np.fromfile(sys.argv[1], dtype=np.uint64)
    off, steps = 0, []
    while off < raw.size:
        n = int(raw[off])
        steps.append(raw[off + 1: off + 1 + n * 8].reshape(n, 8))
        off += 1 + n * 8
    names = ["res", "set", "gather", "decode", "publish"]
    rows = []
    for t in steps:
        t = t.astype(np.int64)
        ok = (t[:, 0] > 0) & (t[:, 5] > 0)
        t = t[ok]
        if not len(t):
            continue
        # phases a workgroup skipped (mode without a set / gather) carry 0: take the last stamp before
        tt = t[:, :6].copy()
        for i in range(1, 6):
            tt[:, i] = np.where(tt[:, i] == 0, tt[:, i - 1], tt[:, i])
        span = (tt[:, 5].max() - tt[:, 0].min()) * 10 / 1e3   # us
        life = (tt[:, 5] - tt[:, 0]) * 10 / 1e3
        ph = [(tt[:, i + 1] - tt[:, i]).mean() * 10 / 1e3 for i in range(5)]
        rows.append([len(t), span, life.mean(), life.sum() / span] + ph)
    a = np.array(rows)
    print(f"{len(a)} steps, {a[:, 0].mean():.0f} workgroups each")
    print(f"kernel span {a[:, 1].mean():.1f} us, workgroup lifetime {a[:, 2].mean():.2f} us, "
          f"in flight {a[:, 3].mean():.0f}")
    for i, nm in enumerate(names):
        print(f"  {nm:<8} {a[:, 4 + i].mean():7.2f} us")


if __name__ == "__main__":
    main()
