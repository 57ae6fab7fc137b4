#!/bin/bash
# Workgroups per CU (capped with PBGPU_LDS_PAD) vs build-kernel time, per config (in-process A/B, scripts/ab_env.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/occ
export REPS=${REPS:-4}
run() { timeout -k 10 150 python3 scripts/ab_env.py "$@" > gpurun_out/occ/$1.jsonl 2>&1 || { cat gpurun_out/occ/$1.jsonl; exit 1; }; cat gpurun_out/occ/$1.jsonl; }
run c2_udp_64 33554432 d: p7:PBGPU_LDS_PAD=5632 p6:PBGPU_LDS_PAD=9728 p5:PBGPU_LDS_PAD=15360 p4:PBGPU_LDS_PAD=23552 p3:PBGPU_LDS_PAD=36864
run c2_udp_1500 8388608 d: p4:PBGPU_LDS_PAD=12352 p3:PBGPU_LDS_PAD=25664 p2:PBGPU_LDS_PAD=53312
run c3_udp_var 8388608 d: p4:PBGPU_LDS_PAD=11672 p3:PBGPU_LDS_PAD=24984
run c4_tcp_syn 33554432 d: p4:PBGPU_LDS_PAD=10496 p3:PBGPU_LDS_PAD=23808
