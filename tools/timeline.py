"""GPU timeline of a serving run (PM_TIMELINE=<file> python bench.py ...:
every timed launch of the kernel-timing pass as kernel,start_us,end_us,ctx).

python tools/timeline.py FILE

Prints per kernel the summed and union time, the time with 0/1/2/... launches
of any kernel running, the answer kernels' concurrency, and the phases
(query phase = before the first prep kernel, maintenance = prep kernels)."""
import collections
import sys

rows = []
for ln in open(sys.argv[1]):
    n, a, b, c = ln.strip().split(",")
    rows.append((float(a), float(b), n, c))
rows.sort()
t0, t1 = rows[0][0], max(r[1] for r in rows)


def union(iv):
    s, ce, cs = 0.0, None, None
    for a, b in sorted(iv):
        if ce is None or a > ce:
            if ce is not None:
                s += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    return s + (ce - cs if ce is not None else 0.0)


def conc(iv, lo, hi):
    ev = []
    for a, b in iv:
        a, b = max(a, lo), min(b, hi)
        if b > a:
            ev += [(a, 1), (b, -1)]
    ev.sort()
    h, c, last = collections.defaultdict(float), 0, lo
    for t, d in ev:
        h[c] += t - last
        c, last = c + d, t
    h[c] += hi - last
    return {k: round(v / 1e3, 2) for k, v in sorted(h.items())}


print(f"span {(t1 - t0) / 1e3:.2f} ms, {len(rows)} launches")
by = collections.defaultdict(list)
for a, b, n, c in rows:
    by[n].append((a, b))
for n, iv in sorted(by.items(), key=lambda x: -sum(b - a for a, b in x[1])):
    print(f"  {n:16s} n={len(iv):5d} sum {sum(b - a for a, b in iv) / 1e3:8.2f} ms  union {union(iv) / 1e3:8.2f} ms  "
          f"avg {sum(b - a for a, b in iv) / len(iv):8.2f} us")
prep = [r for r in rows if r[2].startswith("prep")]
qend = min(r[0] for r in prep) if prep else t1
print(f"query phase {(qend - t0) / 1e3:.2f} ms: any kernel running {conc([(a, b) for a, b, n, c in rows], t0, qend)} ms")
print(f"  answers running {conc(by.get('answer', []), t0, qend)}")
print(f"  match_resolve running {conc(by.get('match_resolve', []), t0, qend)}")
if prep:
    pe = max(r[1] for r in prep)
    print(f"maintenance {(pe - qend) / 1e3:.2f} ms (first prep kernel -> last), prep kernels union "
          f"{union([(a, b) for a, b, n, c in prep]) / 1e3:.2f} ms; after it until the end {(t1 - pe) / 1e3:.2f} ms")
# gaps between consecutive kernels of one team's stream (ctx of the team's steps)
per = collections.defaultdict(list)
for a, b, n, c in rows:
    per[c].append((a, b, n))
for c, v in per.items():
    if len(v) < 100:
        continue
    v.sort()
    gaps = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1) if v[i + 1][2] == "match_resolve" and v[i][2] == "answer"]
    inner = [v[i + 1][0] - v[i][1] for i in range(len(v) - 1) if v[i + 1][2] == "answer" and v[i][2] == "match_resolve"]
    if gaps:
        gaps.sort()
        print(f"  ctx {c}: answer->next match gap median {gaps[len(gaps) // 2]:.1f} us (host round trip), "
              f"match->answer gap median {sorted(inner)[len(inner) // 2]:.1f} us, launches {len(v)}")
