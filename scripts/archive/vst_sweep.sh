#!/bin/bash
# pb_vstage_kernel occupancy sweep on configs[2]: stage KiB x frames per workgroup
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-4} timeout -k 10 400 python3 -u scripts/ab_env.py c3_udp_var 8388608 \
  kb8_w64:PBGPU_STAGE_KB=8,PBGPU_WGF=64 kb8_w128:PBGPU_STAGE_KB=8,PBGPU_WGF=128 \
  kb12_w64:PBGPU_STAGE_KB=12,PBGPU_WGF=64 kb12_w128:PBGPU_STAGE_KB=12,PBGPU_WGF=128 \
  kb16_w64:PBGPU_STAGE_KB=16,PBGPU_WGF=64 kb16_w128:PBGPU_STAGE_KB=16,PBGPU_WGF=128 \
  kb16_w32:PBGPU_STAGE_KB=16,PBGPU_WGF=32 kb12_g16:PBGPU_STAGE_KB=12,PBGPU_G=16 \
  kb8_st:PBGPU_STAGE_KB=8,PBGPU_FST_DBG=1 kb8_co:PBGPU_STAGE_KB=8,PBGPU_FST_DBG=2 \
  stage_kb16:PBGPU_KERNEL=stage,PBGPU_STAGE_KB=16 stage_kb12:PBGPU_KERNEL=stage,PBGPU_STAGE_KB=12 \
  | tee gpurun_out/vst_sweep.txt
