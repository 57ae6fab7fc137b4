#!/bin/bash
# GPF lanes-per-frame sweep over frame lengths with different line alignment,
# plus the write-pattern microbenchmark.  Output under gpurun_out/.
set -e
mkdir -p gpurun_out
for g in ${GS:-8 16 32 64}; do
  PBGPU_G=$g LENS=${LENS:-1500,1504,1536,1024} timeout -k 10 200 python3 scripts/align_probe.py G$g > gpurun_out/glen_G$g.json
done
if [ -x pb-af-xdp_amd/build/wbench ]; then timeout -k 10 120 pb-af-xdp_amd/build/wbench $((3<<30)) > gpurun_out/wbench.txt; fi
cat gpurun_out/glen_G*.json gpurun_out/wbench.txt 2>/dev/null
