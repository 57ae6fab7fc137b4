#!/bin/bash
# pb_xpage_kernel: small-frame parity, then in-process A/B of page counts against the linear small kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -m gpu -k "small or shape or tcp or full_size or golden or oracle" --timeout 120 \
  --timeout-method thread > gpurun_out/xp_par.txt 2>&1 || { tail -40 gpurun_out/xp_par.txt; exit 1; }
tail -n 1 gpurun_out/xp_par.txt
REPS=5 timeout -k 10 300 python3 -u scripts/ab_env.py c4_tcp_syn 33554432 np3: np2:PBGPU_XP_NP=2 np4:PBGPU_XP_NP=4 np7:PBGPU_XP_NP=7 linear:PBGPU_KERNEL=nopage | tee gpurun_out/xp_ab.txt
