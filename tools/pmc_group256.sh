#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the merged maintenance's fold launch shape (256 SIFT1M clients,
# tools/group_fold_probe.py), one pass each.  usage: tools/pmc_group256.sh OUTDIR
out=$GRAFT_REPO_ROOT/$1
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/group_fold_probe.py 256 1"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/f -o run -- $P > $out/f.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/w -o run -- $P > $out/w.log 2>&1 || exit 1
cat $out/f.log
