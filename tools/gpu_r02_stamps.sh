set -o pipefail
F="--steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-bigann --no-config0 --no-single --no-msmarco-search"
rm -f gpurun_out/st_iso.bin gpurun_out/st_con.bin
PM_LIB=build/libpacmann_stamps.so PM_ANSWER_STAMPS=gpurun_out/st_iso.bin timeout -k 10 300 python -u bench.py $F --sessions 64 --groups 1 > gpurun_out/st_iso.json 2>/dev/null || exit 1
PM_LIB=build/libpacmann_stamps.so PM_ANSWER_STAMPS=gpurun_out/st_con.bin timeout -k 10 300 python -u bench.py $F > gpurun_out/st_con.json 2>/dev/null || exit 1
python tools/answer_stamps.py gpurun_out/st_iso.bin && python tools/answer_stamps.py gpurun_out/st_con.bin
gzip -f gpurun_out/st_iso.bin gpurun_out/st_con.bin
