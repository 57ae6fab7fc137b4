#!/bin/bash
# vline (unified chunk path): parity subset, then an alternating A/B against pb_vstage_kernel
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "vline or multi_random or c3_udp_var or counters" -x -q \
    --timeout 120 --timeout-method thread > $O/vline.log 2>&1 || exit 1
REPS=6 timeout -k 10 300 python -u scripts/ab_env.py c3_udp_var 33554432 'vline:' 'vstage:PBGPU_KERNEL=vstage' \
    'vl_pad8k:PBGPU_LDS_PAD=8192' > $O/ab_c3.jsonl 2>&1 || exit 1
