#!/bin/bash
# pb_vstage_kernel: larger windows at 4 workgroups per CU by taking fewer frames per workgroup
# (configs[2], 2^25 frames): default (24 KiB, ~248 frames), 28 KiB with 176, 30 KiB with 128.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/libpbgpu.so
REPS=5 timeout -k 10 300 python3 scripts/ab_lib.py c3_udp_var 33554432 kb24:$L kb28_wgf176:$L:PBGPU_STAGE_KB=28,PBGPU_WGF=176 kb30_wgf128:$L:PBGPU_STAGE_KB=30,PBGPU_WGF=128 > gpurun_out/ab/vst_win_r02c.txt 2>&1; rc=$?
cat gpurun_out/ab/vst_win_r02c.txt; exit $rc
