"""One line per bench JSON (tools/ab.sh): python tools/ab_summary.py sift|bigann LABEL FILE...

sift:   q/s, ms per step and the step / maintenance kernel averages (us), contended and isolated
bigann: per BIGANN block, q/s, ms per round and the step kernel averages (us)
"""
import json
import sys

kind, label = sys.argv[1], sys.argv[2]
for f in sys.argv[3:]:
    d = json.load(open(f))
    if kind == "sift":
        k, iso = d["kernel_avg_us"], (d.get("isolated") or {}).get("kernel_avg_us", {})
        print(label, d["value"], d["ms_per_step"],
              *(f"{n} {k.get(n)}" for n in ("answer", "match_resolve", "prep_fold", "prep_offsets")),
              *(f"iso_{n} {iso.get(n)}" for n in ("answer", "match_resolve")),
              "single_ms", (d.get("single_session") or {}).get("ms_per_query"))
    else:
        for c in ("config3_bigann_100m", "config4_bigann_1b"):
            if c in d:
                x, k = d[c], d[c]["kernel_avg_us"]
                print(label, c, x["private_queries_per_s"], x["ms_per_round"],
                      *(f"{n} {k.get(n)}" for n in ("hint_match", "resolve", "gather", "answer", "l2_rows")))
