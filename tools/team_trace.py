"""Summary of a pooled serving loop's host trace (PM_TEAM_TRACE=<file>, pm_engine.cpp TeamTrace).

python tools/team_trace.py TRACE.csv [t0_ms t1_ms]

Kinds: 0 session task, 1 step launch, 2 maintenance, 3 query start, 4 step in
flight (launch end -> seen complete).  Prints, over the window (default: the
whole trace), the time with 0, 1, 2, ... teams' steps in flight or launching,
the time in maintenance, and per-team phase averages (tasks per open phase,
launch, flight).
"""
import csv
import sys
from collections import defaultdict

rows = [(int(r["team"]), int(r["kind"]), int(r["worker"]), float(r["t0_us"]), float(r["t1_us"]))
        for r in csv.DictReader(open(sys.argv[1]))]
t0 = float(sys.argv[2]) * 1e3 if len(sys.argv) > 2 else min(r[3] for r in rows)
t1 = float(sys.argv[3]) * 1e3 if len(sys.argv) > 3 else max(r[4] for r in rows)
rows = [r for r in rows if r[4] > t0 and r[3] < t1]
span = t1 - t0

# GPU-side occupancy proxy: a team's step from its launch's start to the moment a worker saw it complete
ev = []
for team, kind, w, a, b in rows:
    if kind in (1, 4):
        ev.append((max(a, t0), 1))
        ev.append((min(b, t1), -1))
ev.sort()
hist = defaultdict(float)
cur, last = 0, t0
for t, d in ev:
    hist[cur] += t - last
    cur, last = cur + d, t
hist[cur] += t1 - last
maint = sum(min(b, t1) - max(a, t0) for team, kind, w, a, b in rows if kind == 2)
print(f"window {span / 1e3:.2f} ms; maintenance spans (summed over teams) {maint / 1e3:.2f} ms")
for n in sorted(hist):
    print(f"  {n} teams launching/in flight: {hist[n] / 1e3:8.2f} ms ({hist[n] / span:.1%})")

per = defaultdict(list)
for team, kind, w, a, b in rows:
    per[kind].append(b - a)
names = {0: "session task", 1: "step launch", 2: "maintenance", 3: "query start", 4: "step in flight"}
for kind in sorted(per):
    v = per[kind]
    print(f"  {names.get(kind, kind):15s} n={len(v):6d} mean {sum(v) / len(v):8.1f} us, total {sum(v) / 1e3:8.2f} ms")
workers = {w for team, kind, w, a, b in rows if kind == 0}
busy = sum(b - a for team, kind, w, a, b in rows if kind in (0, 1, 3))
print(f"  host busy (tasks + launches + starts) {busy / 1e3:.2f} ms over {len(workers)} workers "
      f"= {busy / span / max(1, len(workers)):.1%} of their time")
