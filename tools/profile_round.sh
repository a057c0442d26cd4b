#!/bin/bash
# Round profile set (run on the GPU box from the repo root):
#   bench line, kernel stats and the two PMC passes of the same bench command
#   (SIFT1M sessions + the BIGANN-100M / 1B blocks).
# usage: tools/profile_round.sh OUTDIR
set -e
out=$1; mkdir -p "$out"
export TMPDIR=/tmp
cmd="bench.py --steps 30 --warmup 1 --no-cpu-baseline --no-config2 --no-config0 --no-single"
timeout -k 10 400 python3 -u bench.py --steps 200 --warmup 5 > "$out/bench.json" 2> "$out/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/ks" -o run -- python3 $cmd > "$out/ks.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pf" -o run -- python3 $cmd > "$out/pf.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pw" -o run -- python3 $cmd > "$out/pw.log" 2>&1
echo done
