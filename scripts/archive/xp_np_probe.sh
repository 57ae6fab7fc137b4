#!/bin/bash
# pb_xpage_kernel for frames > 64 B: pages per workgroup that fill one pass of lanes, against the linear kernel
set -o pipefail
mkdir -p gpurun_out
XP_EXTRA="np4:PBGPU_XP_FORCE=1,PBGPU_XP_NP=4 np5:PBGPU_XP_FORCE=1,PBGPU_XP_NP=5 np6:PBGPU_XP_FORCE=1,PBGPU_XP_NP=6 w512np8:PBGPU_XP_FORCE=1,PBGPU_XP_WGT=512,PBGPU_XP_NP=8 w512np11:PBGPU_XP_FORCE=1,PBGPU_XP_WGT=512,PBGPU_XP_NP=11" \
XP_CASES="c5_icmp_echo c1_udp_static_106 c2_udp_64:100 c2_udp_64:72" REPS=3 timeout -k 10 400 python3 -u scripts/xp_len_ab.py | tee gpurun_out/xpn_ab.txt
