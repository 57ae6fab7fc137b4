#!/bin/bash
# Round 3: re-tune the staged 1500-B kernel and the 2-mod-4 small kernel now that both write
# XCD-contiguous regions (shapes picked in rounds 1-2 without them).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2l}
mkdir -p $O
REPS=6 timeout -k 10 400 python -u scripts/ab_env.py c2_udp_1500 33554432 'wgf64:' 'wgf32:PBGPU_FST_WGF=32' \
    'wgf128:PBGPU_FST_WGF=128' 'nbuf2:PBGPU_FST_NBUF=2' 'g32:PBGPU_FST_G=32' > $O/ab_1500_shape.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 240 python -u scripts/ab_env.py c5_icmp_echo 33554432 'wgt64:' 'wgt128:PBGPU_SMALL_WGT=128' \
    'wgt256:PBGPU_SMALL_WGT=256' > $O/ab_icmp98_wgt.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 240 python -u scripts/ab_env.py c2_udp_64 33554432 'occ8:' 'occ6:PBGPU_LDS_PAD=10000' \
    'occ4:PBGPU_LDS_PAD=24000' > $O/ab_udp64_occ.jsonl 2>&1 || exit 1
