#!/bin/bash
# adaptive lanes per frame vs fixed 8-lane groups, configs[2] at the bench size, more repetitions
set -o pipefail
mkdir -p gpurun_out
REPS=${REPS:-6} timeout -k 10 500 python3 -u scripts/ab_env.py c3_udp_var 16777216 \
  adapt: fixed8:PBGPU_FST_DBG=16 adapt_kb20:PBGPU_STAGE_KB=20 fixed8_kb20:PBGPU_FST_DBG=16,PBGPU_STAGE_KB=20 adapt_kb18:PBGPU_STAGE_KB=18 \
  | tee gpurun_out/va_ab2.txt
