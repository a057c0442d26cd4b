#!/bin/bash
# Same-box ABBA A/B of an environment switch on the SIFT1M serving line
# (headline block only).  usage: tools/ab_env_bench.sh OUTDIR VAR VALUE_A VALUE_B [bench args]
out=$1; var=$2; a=$3; b=$4; shift 4
mkdir -p $out
args=${*:---steps 40 --warmup 3}
for v in $a $b $b $a; do
  env $var=$v timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-config2 --no-msmarco-search \
    --no-config0 --no-bigann > $out/${var}_$v.$RANDOM.json 2>> $out/err.log || exit 1
done
python3 - $out <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    k = d["kernel_avg_us"]; iso = d.get("isolated", {}).get("kernel_avg_us", {})
    print(os.path.basename(f), d["value"], "answer", k["answer"], "iso", iso.get("answer"), "mr", k["match_resolve"],
          "fold", k["prep_fold"], "offs", k["prep_offsets"])
PY
