#!/bin/bash
# diagnostic: store-only pb_fstage_kernel, linear vs XCD-owned 4 KiB page stores, by frames per workgroup
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-5} timeout -k 10 300 python3 -u scripts/ab_env.py c2_udp_1500 8388608 \
  lin_w16:PBGPU_FST_G=16,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=9,PBGPU_FST_WGF=16 \
  xcd_w16:PBGPU_FST_G=16,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=15,PBGPU_FST_WGF=16 \
  xcd_w32:PBGPU_FST_G=16,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=15,PBGPU_FST_WGF=32 \
  xcd_w64:PBGPU_FST_G=16,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=15,PBGPU_FST_WGF=64 \
  xcd_g32_w8:PBGPU_FST_G=32,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=15,PBGPU_FST_WGF=8 \
  lin_g32_w8:PBGPU_FST_G=32,PBGPU_FST_NBUF=1,PBGPU_FST_DBG=9,PBGPU_FST_WGF=8 \
  | tee gpurun_out/fst_xcd.txt
