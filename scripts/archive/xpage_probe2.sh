#!/bin/bash
# pb_xpage_kernel page-count sweep: 60-B TCP and (forced) 64-B UDP against their defaults
set -o pipefail
mkdir -p gpurun_out
REPS=5 timeout -k 10 300 python3 -u scripts/ab_env.py c4_tcp_syn 33554432 np7:PBGPU_XP_NP=7 np10:PBGPU_XP_NP=10 np11:PBGPU_XP_NP=11 np14:PBGPU_XP_NP=14 np15:PBGPU_XP_NP=15 linear:PBGPU_KERNEL=nopage | tee gpurun_out/xp_ab2.txt
REPS=5 timeout -k 10 300 python3 -u scripts/ab_env.py c2_udp_64 33554432 xsmall: xp4:PBGPU_XP_FORCE=1,PBGPU_XP_NP=4 xp8:PBGPU_XP_FORCE=1,PBGPU_XP_NP=8 xp12:PBGPU_XP_FORCE=1,PBGPU_XP_NP=12 xp15:PBGPU_XP_FORCE=1,PBGPU_XP_NP=15 | tee -a gpurun_out/xp_ab2.txt
