#!/bin/bash
# SQ counters of the preprocessing kernels (tools/fold_probe.py): VALU / LDS activity
mkdir -p gpurun_out/pmc_prep
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d $GRAFT_REPO_ROOT/gpurun_out/pmc_prep/a -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fold_probe.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_prep/a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/pmc_prep/b -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fold_probe.py > $GRAFT_REPO_ROOT/gpurun_out/pmc_prep/b.log 2>&1 || exit 1
echo done
