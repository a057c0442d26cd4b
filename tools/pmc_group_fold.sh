#!/bin/bash
# SQ / TCC counters of the 64-client group fold (tools/group_fold_probe.py), one pass each.
# usage: tools/pmc_group_fold.sh OUTDIR [LIB]
out=$GRAFT_REPO_ROOT/$1
mkdir -p $out
[ -n "$2" ] && export PM_LIB=$GRAFT_REPO_ROOT/$2
cd /tmp && export TMPDIR=/tmp
P="python3 $GRAFT_REPO_ROOT/tools/group_fold_probe.py 64 2"
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d $out/a -o pmc --output-format csv -- $P > $out/a.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE -d $out/b -o pmc --output-format csv -- $P > $out/b.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $out/c -o pmc --output-format csv -- $P > $out/c.log 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $out/d -o pmc --output-format csv -- $P > $out/d.log 2>&1 || exit 1
echo done
