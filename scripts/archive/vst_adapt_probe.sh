#!/bin/bash
# pb_vstage_kernel with 32 / 16 / 8 lanes per frame by window (every lane busy): parity, then A/B
# against the fixed 8-lane groups (PBGPU_FST_DBG=16) on configs[2] and odd fixed lengths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -m gpu -k "vstage or variable or var or c3" --timeout 120 \
  --timeout-method thread > gpurun_out/va_par.txt 2>&1 || { tail -40 gpurun_out/va_par.txt; exit 1; }
tail -n 1 gpurun_out/va_par.txt
REPS=${REPS:-4} timeout -k 10 400 python3 -u scripts/ab_env.py c3_udp_var 8388608 \
  adapt: fixed8:PBGPU_FST_DBG=16 no32:PBGPU_FST_DBG=32 adapt_kb24:PBGPU_STAGE_KB=24 fixed8_kb24:PBGPU_FST_DBG=16,PBGPU_STAGE_KB=24 \
  adapt_kb12:PBGPU_STAGE_KB=12 adapt_w96:PBGPU_WGF=96 adapt_kb20:PBGPU_STAGE_KB=20 \
  | tee gpurun_out/va_ab.txt
