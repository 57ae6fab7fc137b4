#!/bin/bash
# pb_fstage_kernel time decomposition (diagnostic switches, wrong output):
# full / store-only (no payload) / compute-only (no stores) / phase A only
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-5} timeout -k 10 300 python3 -u scripts/ab_env.py ${CFG:-c2_udp_1500} ${NPK:-8388608} \
  full:PBGPU_FST_G=${G:-16} \
  store_only:PBGPU_FST_G=${G:-16},PBGPU_FST_DBG=1 \
  compute_only:PBGPU_FST_G=${G:-16},PBGPU_FST_DBG=2 \
  a_only:PBGPU_FST_G=${G:-16},PBGPU_FST_DBG=3 \
  stage:PBGPU_KERNEL=stage \
  | tee gpurun_out/fst_decomp.txt
