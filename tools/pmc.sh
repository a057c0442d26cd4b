#!/bin/bash
# rocprofv3 counter passes over one program, one pass per counter set (at most
# 8 SQ_ / 4 TCC_ counters each; FETCH_SIZE alone, WRITE_SIZE alone), each under
# its own kill-timer.  Run from the repo root through gpurun.
#
# usage: tools/pmc.sh OUTDIR SETS -- PROGRAM ARGS...
#   SETS  hbm       FETCH_SIZE | WRITE_SIZE            (tools/pmc_summary.py reads these)
#         lds       SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES
#                   SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS
#         valu      SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM
#                   SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE
#         comma-separated: e.g. hbm,lds
# e.g. tools/pmc.sh gpurun_out/pmc_fold hbm,lds -- python3 tools/group_fold_probe.py 64 2
out=$GRAFT_REPO_ROOT/$1; sets=$2; shift 2
[ "$1" = "--" ] && shift
mkdir -p "$out"
prog=("$@")
[ "${prog[1]#/}" = "${prog[1]}" ] && [ -e "${prog[1]}" ] && prog[1]=$GRAFT_REPO_ROOT/${prog[1]}   # script path
cd /tmp && export TMPDIR=/tmp
pass() {   # NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o pmc -- "${prog[@]}" \
    > "$out/$name.log" 2>&1 || { echo "pass $name failed"; tail -5 "$out/$name.log"; exit 1; }
}
IFS=, read -ra S <<< "$sets"
for s in "${S[@]}"; do
  case $s in
    hbm) pass fetch FETCH_SIZE && pass write WRITE_SIZE ;;
    lds) pass lds SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
           SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS ;;
    valu) pass valu SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM \
            SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE ;;
    *) echo "unknown set $s"; exit 2 ;;
  esac
done
find "$out" -name "*.csv" -size +1M -exec gzip -f {} \;
echo done
