#!/bin/bash
# pb_vline_kernel shape A/B on configs[2] (2^25 frames): frames per workgroup (region size) and
# occupancy (PBGPU_LDS_PAD adds LDS per workgroup: 5 -> 4 -> 3 workgroups per CU)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03f}
mkdir -p $O
REPS=${REPS:-3} timeout -k 10 400 python -u scripts/ab_env.py c3_udp_var 33554432 'w252:' 'w192:PBGPU_VL_WGF=192' \
    'w128:PBGPU_VL_WGF=128' 'w64:PBGPU_VL_WGF=64' 'w32:PBGPU_VL_WGF=32' 'occ4:PBGPU_LDS_PAD=8192' \
    'occ3:PBGPU_LDS_PAD=26000' 'w128nogen:PBGPU_VL_WGF=128,PBGPU_FST_DBG=1' 'w252nogen:PBGPU_FST_DBG=1' \
    > $O/ab.jsonl 2>&1 || exit 1
