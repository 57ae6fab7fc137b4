#!/bin/bash
# pb_vstage_kernel: line-aligned workgroup edges (ghost frames) vs the round-1 split edges (PBGPU_FST_DBG=64)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/vedge
export REPS=${REPS:-8}
timeout -k 10 250 python3 scripts/ab_env.py c3_udp_var 16777216 lines: split:PBGPU_FST_DBG=64 > gpurun_out/vedge/c3.jsonl 2>&1 || { cat gpurun_out/vedge/c3.jsonl; exit 1; }
cat gpurun_out/vedge/c3.jsonl
timeout -k 10 250 python3 scripts/ab_env.py udp_fixed_odd_65 33554432 lines: split:PBGPU_FST_DBG=64 > gpurun_out/vedge/odd65.jsonl 2>&1 || { cat gpurun_out/vedge/odd65.jsonl; exit 1; }
cat gpurun_out/vedge/odd65.jsonl
