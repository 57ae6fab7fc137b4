#!/bin/bash
# pb_vstage_kernel on configs[2]: frames per workgroup below one window's worth of
# minimum-length frames (PBGPU_WGF now authoritative) x stage KiB
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "vstage or variable or var" --timeout 120 \
  --timeout-method thread > gpurun_out/vw_par.txt 2>&1 || { tail -40 gpurun_out/vw_par.txt; exit 1; }
tail -n 1 gpurun_out/vw_par.txt
REPS=${REPS:-4} timeout -k 10 500 python3 -u scripts/ab_env.py c3_udp_var 8388608 \
  base: w32:PBGPU_WGF=32 w48:PBGPU_WGF=48 w64:PBGPU_WGF=64 w96:PBGPU_WGF=96 \
  w64_kb12:PBGPU_WGF=64,PBGPU_STAGE_KB=12 w64_kb20:PBGPU_WGF=64,PBGPU_STAGE_KB=20 w64_kb24:PBGPU_WGF=64,PBGPU_STAGE_KB=24 \
  w96_kb24:PBGPU_WGF=96,PBGPU_STAGE_KB=24 w48_kb20:PBGPU_WGF=48,PBGPU_STAGE_KB=20 \
  | tee gpurun_out/vw_sweep.txt
