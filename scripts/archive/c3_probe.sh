#!/bin/bash
# configs[2] (packed variable lengths): whole step (length passes + build) vs build kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 3 --no-variants --cpu-seconds 0 --config c3_udp_var \
  --packets 16777216 > gpurun_out/c3_bench.txt 2>&1 || { tail -20 gpurun_out/c3_bench.txt; exit 1; }
cat gpurun_out/c3_bench.txt
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-variants --cpu-seconds 0 --ramp-seconds 0.2 --config c3_udp_var --packets 16777216 > gpurun_out/c3_prof.log 2>&1 || { tail -20 gpurun_out/c3_prof.log; exit 1; }
cat gpurun_out/c3_prof/run_kernel_stats.csv
