"""One line per bench JSON: q/s and the step / maintenance kernel averages (us), contended and isolated."""
import json
import sys

for f in sys.argv[1:]:
    d = json.load(open(f))
    k, iso = d["kernel_avg_us"], d["isolated"]["kernel_avg_us"]
    print(f, d["value"], *(f"{n} {k.get(n)}" for n in ("answer", "match_resolve", "prep_fold", "prep_offsets")),
          *(f"iso_{n} {iso.get(n)}" for n in ("answer", "match_resolve", "prep_fold_one_client", "prep_offsets_one_client")))
