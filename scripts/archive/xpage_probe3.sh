#!/bin/bash
# pb_xpage_kernel default shape: full GPU suite, then A/B against the linear small kernel at several lengths
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/xp_full.txt 2>&1 || { tail -40 gpurun_out/xp_full.txt; exit 1; }
tail -n 1 gpurun_out/xp_full.txt
REPS=5 timeout -k 10 300 python3 -u scripts/ab_env.py c4_tcp_syn 33554432 xpage: linear:PBGPU_KERNEL=nopage | tee gpurun_out/xp_ab3.txt
timeout -k 10 300 python3 -u scripts/len_ab.py | tee -a gpurun_out/xp_ab3.txt
