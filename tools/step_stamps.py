"""Diagnostic: where a fused k_step spends its time.

Build the PM_STEP_STAMPS variant here (it travels with the snapshot):
    python tools/step_stamps.py --build
then on the GPU box:
    PM_LIB=pacmann_amd/libpacmann_ststamps.so PM_STAMP_FILE=gpurun_out/st.bin \\
        python tools/step_stamps.py --run && python tools/step_stamps.py --show gpurun_out/st.bin
Stamps are s_memrealtime (100 MHz) per workgroup: 0 start, 1 (match: role
end; answer: guess done), 2 end; 3: XCC_ID << 32 | HW_ID (answer: resolution
seen << 1 | guess kept).  Workgroups: nsub match, np resolvers, nsub answers.
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


def run(steps=300, c2=False):
    import pacmann_amd as pm
    # default: SIFT1M-sized rounds of 96 ids; --c2: bench.py's configs[2]
    # TestBatchPIRPerf shape (3,201,821 x 896 B, batches of 32 ids)
    N, E, B, ids = (3_201_821, 112, 32, 32) if c2 else (1_000_000, 80, 32, 96)
    db = np.random.default_rng(0).integers(0, 2**64, size=N * E, dtype=np.uint64)
    g = pm.SimpleBatchPianoPIR(N, E * 8, B, db, 8, seed=1)
    g.Preprocessing()
    rng = np.random.default_rng(1)
    for q in rng.integers(0, N, size=(steps, ids)).astype(np.uint64):
        g.Query(q)


def show(fn):
    raw = np.fromfile(fn, dtype=np.uint8)
    off, rows = 0, []
    while off < raw.size:
        grid, nsub, cblk, np_ = raw[off:off + 16].view(np.uint32)
        off += 16
        t8 = raw[off:off + grid * 64].view(np.uint64)
        off += grid * 64
        t, ms = t8[:grid * 4].reshape(grid, 4), t8[grid * 4:].reshape(grid, 4)
        t0 = t[:, 0][t[:, 0] > 0].min()
        rel = np.where(t[:, :3] > 0, t[:, :3].astype(np.int64) - t0, -1) * 10 / 1000.0   # us
        a0 = grid - nsub   # answers last (after nhelp x nsub gather helpers, if any)
        m, r, a = rel[:nsub], rel[nsub:nsub + np_], rel[a0:]
        live = r[:, 0] >= 0
        seen = t[a0:, 3]
        a_seen = ((seen >> 1).astype(np.int64) - int(t0)) * 0.01
        kept = (seen & 1).astype(bool)
        arel = (ms[a0:, :2].astype(np.int64) - int(t0)) * 0.01
        okr = ms[a0:, 0] > 0
        hp = rel[nsub + np_:a0]   # gather helpers (start, -, end)
        hl = [np.median(hp[:, 2]), hp[:, 2].max()] if len(hp) else [0.0, 0.0]
        rows.append([*hl, np.median(arel[okr, 0]), arel[okr, 0].max(), np.median(arel[okr, 1]), arel[okr, 1].max(),
                     m[:, 0].max(), np.median(m[:, 1]), m[:, 1].max(),
                     np.median(r[live, 2]), r[live, 2].max(),
                     a[:, 1].max(), a_seen.max(), np.median((a[:, 2] - a_seen)[kept]) if kept.any() else 0,
                     np.median((a[:, 2] - a_seen)[~kept]) if (~kept).any() else 0, kept.mean(), a[:, 2].max()])
    rows = np.array(rows[10:])
    names = ["helper median end", "helper last end", "answer median scan done", "answer last scan done", "answer median set done",
             "answer last set done", "match last start", "match median role end", "match last role end",
             "resolver median end", "resolver last end", "answer last guess done",
             "answer last result seen", "answer after result, kept", "answer after result, redone",
             "answer fraction kept", "answer last end"]
    print(f"{len(rows)} steps; us since the first workgroup start (median / p10 / p90)")
    for i, n in enumerate(names):
        print(f"  {n:26s} {np.median(rows[:, i]):7.2f} {np.percentile(rows[:, i], 10):7.2f} "
              f"{np.percentile(rows[:, i], 90):7.2f}")


if __name__ == "__main__":
    if "--build" in sys.argv:
        build()
    if "--run" in sys.argv:
        run(c2="--c2" in sys.argv)
    if "--show" in sys.argv:
        show(sys.argv[sys.argv.index("--show") + 1])
