# k_step gather helpers on/off on one box: phase stamps, then the batch loop's
# timings (tools/batchpir_host.py) in ABBA order
out=${1:-gpurun_out/help5}; mkdir -p $out
for h in 3 0; do
  PM_STEP_HELP=$h PM_LIB=pacmann_amd/libpacmann_ststamps.so PM_STAMP_FILE=$out/c2_h$h.bin timeout -k 10 300 python -u tools/step_stamps.py --run --c2 > $out/run_h$h.log 2>&1 || exit 1
  python tools/step_stamps.py --show $out/c2_h$h.bin > $out/show_h$h.txt 2>&1
done
for h in 0 3 3 0; do
  echo "== PM_STEP_HELP=$h" >> $out/host.log
  PM_STEP_HELP=$h timeout -k 10 300 python -u tools/batchpir_host.py 300 >> $out/host.log 2>&1 || exit 1
done
