#!/bin/bash
# compile-time A/B probes (scripts/ab_lib.py) on the 1500-B and configs[2] kernels
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
export REPS=${REPS:-6}
T=${AB_TAG:-ab}
V=${AB_VARIANTS:-"base:pb-af-xdp_amd/lib/libpbgpu.so ilp:pb-af-xdp_amd/lib/variants/libpbgpu_ilp.so"}
for c in ${AB_CONFIGS:-c2_udp_1500:8388608 c3_udp_var:8388608}; do
  cfg=${c%%:*}; n=${c#*:}
  timeout -k 10 240 python3 -u scripts/ab_lib.py $cfg $n $V > gpurun_out/ab/${T}_$cfg.jsonl 2>&1 || { cat gpurun_out/ab/${T}_$cfg.jsonl; exit 1; }
  cat gpurun_out/ab/${T}_$cfg.jsonl
done
