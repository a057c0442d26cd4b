"""Per-round critical path of the pooled serving loop from its host trace
(PM_TEAM_TRACE=<file>; pm_engine.cpp TeamTrace).

python tools/team_rounds.py TRACE.csv

For every step of every team: the step seen complete (end of its flight
record) -> the first session task of the open phase (pickup), -> the last task
done (open span; tasks, workers and summed task time), -> the launch done
(launch), -> the next completion seen (flight: GPU queueing + kernels +
detection).  Prints medians and means over the rounds of the query phase."""
import csv
import statistics as st
import sys
from collections import defaultdict

rows = [(int(r["team"]), int(r["kind"]), int(r["worker"]), float(r["t0_us"]), float(r["t1_us"]))
        for r in csv.DictReader(open(sys.argv[1]))]
by = defaultdict(lambda: defaultdict(list))
for team, kind, w, a, b in rows:
    by[team][kind].append((a, b, w))
out = defaultdict(list)
for team, k in by.items():
    tasks = sorted(k[0])
    launches = sorted(k[1])
    flights = sorted(k[4], key=lambda x: x[1])
    ti = 0
    for fa, fb, fw in flights:   # fb: the step seen complete
        nxt = [l for l in launches if l[0] >= fb]
        if not nxt:
            continue
        la, lb, lw = nxt[0]
        ph = [t for t in tasks if fb <= t[0] <= la]
        if not ph:
            continue
        nf = [f for f in flights if f[0] >= lb - 1e-6]
        if not nf:
            continue
        out["pickup"].append(ph[0][0] - fb)
        out["open_span"].append(max(t[1] for t in ph) - ph[0][0])
        out["tasks"].append(len(ph))
        out["workers"].append(len({t[2] for t in ph}))
        out["task_us"].append(st.mean(t[1] - t[0] for t in ph))
        out["last_task_to_launch_end"].append(lb - max(t[1] for t in ph))
        out["flight"].append(nf[0][1] - nf[0][0])
        out["cycle"].append(nf[0][1] - fb)
for k, v in out.items():
    print(f"{k:24s} median {st.median(v):8.1f}  mean {st.mean(v):8.1f}  n={len(v)}")
