"""Diagnostic: where a fused k_step spends its time.

Build the PM_STEP_STAMPS variant here (it travels with the snapshot):
    python tools/step_stamps.py --build
then on the GPU box:
    PM_LIB=pacmann_amd/libpacmann_ststamps.so PM_STAMP_FILE=gpurun_out/st.bin \\
        python tools/step_stamps.py --run && python tools/step_stamps.py --show gpurun_out/st.bin
Stamps are s_memrealtime (100 MHz) per workgroup: 0 start, 1 after its wait
(match: after the role), 2 end; 3: XCC_ID << 32 | HW_ID.  Workgroups: nsub
match, np resolvers, nsub answers.
"""
import os
import subprocess
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def build():
    from pacmann_amd import build as B
    out = B.PKG / "libpacmann_ststamps.so"
    cmd = [B.HIPCC, *B.FLAGS, "-DPM_STEP_STAMPS", "-o", str(out), *map(str, B.SOURCES)]
    subprocess.run(cmd, check=True, cwd=B.CSRC)
    print(out)


def run(steps=300):
    import pacmann_amd as pm
    N, E, B = 1_000_000, 80, 32
    db = np.random.default_rng(0).integers(0, 2**64, size=N * E, dtype=np.uint64)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=1)
    g.Preprocessing()
    rng = np.random.default_rng(1)
    for q in rng.integers(0, N, size=(steps, 96)).astype(np.uint64):
        g.Query(q)


def show(fn):
    raw = np.fromfile(fn, dtype=np.uint8)
    off, rows = 0, []
    while off < raw.size:
        grid, nsub, cblk, np_ = raw[off:off + 16].view(np.uint32)
        off += 16
        t = raw[off:off + grid * 32].view(np.uint64).reshape(grid, 4)
        off += grid * 32
        t0 = t[:, 0][t[:, 0] > 0].min()
        rel = np.where(t[:, :3] > 0, t[:, :3].astype(np.int64) - t0, -1) * 10 / 1000.0   # us
        m, r, a = rel[:nsub], rel[nsub:nsub + np_], rel[nsub + np_:]
        live = r[:, 0] >= 0
        rows.append([m[:, 0].max(), np.median(m[:, 1]), m[:, 1].max(), m[:, 2].max(),
                     r[live, 1].max(), np.median(r[live, 2] - r[live, 1]), r[live, 2].max(),
                     a[:, 1].max(), np.median(a[:, 2] - a[:, 1]), a[:, 2].max()])
    rows = np.array(rows[10:])
    names = ["match last start", "match median role end", "match last role end", "match last counted",
             "resolver last poll done", "resolver median body", "resolver last end", "answer last poll done",
             "answer median body", "answer last end"]
    print(f"{len(rows)} steps; us since the first workgroup start (median / p10 / p90)")
    for i, n in enumerate(names):
        print(f"  {n:26s} {np.median(rows[:, i]):7.2f} {np.percentile(rows[:, i], 10):7.2f} "
              f"{np.percentile(rows[:, i], 90):7.2f}")


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    if "--run" in sys.argv:
        run()
    if "--show" in sys.argv:
        show(sys.argv[sys.argv.index("--show") + 1])
