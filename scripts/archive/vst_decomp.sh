#!/bin/bash
# pb_vstage_kernel time decomposition on configs[2] (diagnostic switches, wrong output)
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-5} timeout -k 10 300 python3 -u scripts/ab_env.py c3_udp_var 8388608 \
  full: store_only:PBGPU_FST_DBG=1 compute_only:PBGPU_FST_DBG=2 a_s_only:PBGPU_FST_DBG=3 \
  wgf256:PBGPU_WGF=256 kb16:PBGPU_STAGE_KB=16 kb36:PBGPU_STAGE_KB=36 stage8:PBGPU_KERNEL=stage \
  | tee gpurun_out/vst_decomp.txt
