#!/bin/bash
# after removing the scratch spill: full GPU tests, staged-kernel timings, WRITE_SIZE of the 1500-B build
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sc_par.txt 2>&1 || { tail -40 gpurun_out/sc_par.txt; exit 1; }
tail -n 1 gpurun_out/sc_par.txt
REPS=4 timeout -k 10 300 python3 -u scripts/ab_env.py c2_udp_1500 8388608 fst: | tee gpurun_out/sc_ab.txt
REPS=4 timeout -k 10 300 python3 -u scripts/ab_env.py c3_udp_var 8388608 vst: | tee -a gpurun_out/sc_ab.txt
rm -rf gpurun_out/sc_pmc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sc_pmc -o run -- python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config c2_udp_1500 --packets 8388608 > gpurun_out/sc_pmc.log 2>&1 || { tail -5 gpurun_out/sc_pmc.log; exit 1; }
python3 - <<'PY'
import csv
v=[float(r["Counter_Value"]) for r in csv.DictReader(open("gpurun_out/sc_pmc/run_counter_collection.csv")) if "fstage" in r["Kernel_Name"]]
print("fstage WRITE_SIZE*1024 per launch", sum(v)/len(v)*1024, "algorithmic", 8388608*1500)
PY
