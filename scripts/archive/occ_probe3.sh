#!/bin/bash
# Round 2: confirm the window size of pb_vstage_kernel and the 6-per-CU cap of pb_xsmall_kernel (ab_env.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/occ3
export REPS=${REPS:-8}
run() { tag=$1; shift; timeout -k 10 250 python3 scripts/ab_env.py "$@" > gpurun_out/occ3/$tag.jsonl 2>&1 || { cat gpurun_out/occ3/$tag.jsonl; exit 1; }; echo "== $tag"; cat gpurun_out/occ3/$tag.jsonl; }
run var c3_udp_var 16777216 d: kb18:PBGPU_STAGE_KB=18 kb20:PBGPU_STAGE_KB=20 kb22:PBGPU_STAGE_KB=22 kb24:PBGPU_STAGE_KB=24
run x64 c2_udp_64 33554432 d: p6:PBGPU_LDS_PAD=9728 p7:PBGPU_LDS_PAD=5632
run tcp c4_tcp_syn 33554432 d: p6:PBGPU_LDS_PAD=2048
