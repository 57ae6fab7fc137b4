#!/bin/bash
# Write-roofline shape search + address-map probes (probes/wbench.hip), round 2.
# One file per section under gpurun_out/wbench/ (committed as profiles/r02/wbench/).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wbench
SZ=${WB_SIZE:-2147483648}
for sec in ${WB_SECTIONS:-shapes memset occ paced sparse stride win win2 fown}; do
  timeout -k 10 240 pb-af-xdp_amd/bin/wbench $SZ $sec > gpurun_out/wbench/${sec}_$SZ.txt 2>&1 || { tail -5 gpurun_out/wbench/${sec}_$SZ.txt; exit 1; }
  echo "== $sec"; cat gpurun_out/wbench/${sec}_$SZ.txt
done
