#!/bin/bash
# Round 2 shape A/B of the shipped kernels (scripts/ab_env.py, in-process, alternating):
# workgroups per CU capped with PBGPU_LDS_PAD, fixed-length stage frames per workgroup.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/occ2
export REPS=${REPS:-6}
run() { tag=$1; shift; timeout -k 10 200 python3 scripts/ab_env.py "$@" > gpurun_out/occ2/$tag.jsonl 2>&1 || { cat gpurun_out/occ2/$tag.jsonl; exit 1; }; echo "== $tag"; cat gpurun_out/occ2/$tag.jsonl; }
# pb_xsmall_kernel: 17408 B static LDS, 94 SGPRs (7 workgroups / CU by SGPRs)
run x64 c2_udp_64 33554432 d: p6:PBGPU_LDS_PAD=9728 p5:PBGPU_LDS_PAD=15360 d2: p6b:PBGPU_LDS_PAD=9728
# pb_fstage_kernel: frames per workgroup and 4 / 3 workgroups per CU
run f1500 c2_udp_1500 8388608 d: w16:PBGPU_FST_WGF=16 w32:PBGPU_FST_WGF=32 w128:PBGPU_FST_WGF=128 p4:PBGPU_LDS_PAD=12352
# pb_vstage_kernel: window size
run var c3_udp_var 8388608 d: kb12:PBGPU_STAGE_KB=12 kb20:PBGPU_STAGE_KB=20 p4:PBGPU_LDS_PAD=11672
