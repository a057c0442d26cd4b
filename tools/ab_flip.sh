set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "prf or preprocessing or batch_pir or bigann_partition or group" > gpurun_out/t_fold.log 2>&1 || { echo TESTFAIL; exit 1; }
for i in 1 2; do
  timeout -k 10 120 python -u tools/fold_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit 1
  PM_LIB=$PWD/var/libpacmann_noflip.so timeout -k 10 120 python -u tools/fold_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/lpmc/flip -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fold_probe.py > $GRAFT_REPO_ROOT/gpurun_out/lpmc_flip.log 2>&1 || exit 1
PM_LIB=$GRAFT_REPO_ROOT/var/libpacmann_noflip.so timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $GRAFT_REPO_ROOT/gpurun_out/lpmc/noflip -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/fold_probe.py > $GRAFT_REPO_ROOT/gpurun_out/lpmc_noflip.log 2>&1 || exit 1
echo done
