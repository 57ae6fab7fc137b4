#!/bin/bash
# Write-roofline shape search + address-map probe (tools/wbench.hip), round 2.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wbench
for sz in ${WB_SIZES:-2147483648}; do
  timeout -k 10 240 pb-af-xdp_amd/bin/wbench $sz ${WB_SECTIONS:-} > gpurun_out/wbench/wbench_$sz.txt 2>&1 || { tail -5 gpurun_out/wbench/wbench_$sz.txt; exit 1; }
done
cat gpurun_out/wbench/wbench_*.txt
