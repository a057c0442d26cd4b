#!/bin/bash
# BIGANN-shaped preprocessing kernels: device times (tools/fold_wide_probe.py),
# rocprof kernel stats and HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes).
out=${1:-gpurun_out/foldprobe}; mkdir -p $out
for s in 100m 1b; do timeout -k 10 300 python tools/fold_wide_probe.py $s 2 >> $out/probe.log 2>&1 || exit 1; done
cat $out/probe.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$out/trace -o fw --output-format csv -- python3 $R/tools/fold_wide_probe.py 100m 2 > $R/$out/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/$out/pmc_fetch -o pmc --output-format csv -- python3 $R/tools/fold_wide_probe.py 100m 1 > $R/$out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/$out/pmc_write -o pmc --output-format csv -- python3 $R/tools/fold_wide_probe.py 100m 1 > $R/$out/pmc_write.log 2>&1 || exit 1
echo done
