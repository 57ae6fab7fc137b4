#!/bin/bash
# pb_vstage_kernel: parity (kernel-shape tests + parity suite), then in-process A/B vs pb_stage_kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 \
  --timeout-method thread > gpurun_out/vst_par.txt 2>&1 || { tail -40 gpurun_out/vst_par.txt; exit 1; }
tail -n 2 gpurun_out/vst_par.txt
[ -n "$PARITY_ONLY" ] && exit 0
REPS=${REPS:-5} timeout -k 10 300 python3 -u scripts/ab_env.py c3_udp_var 8388608 \
  stage8:PBGPU_KERNEL=stage vst8: vst16:PBGPU_G=16 stage16:PBGPU_KERNEL=stage,PBGPU_G=16 \
  | tee gpurun_out/vst_ab.txt
