#!/bin/bash
# pb_vstage_kernel window size vs workgroups per CU, end of round 2 (configs[2], 2^25 frames):
# the default 24 KiB window (4 per CU), 20 KiB (4 per CU), 16 KiB with 240 frames per
# workgroup (5 per CU), 12 KiB with 226 (6 per CU).  Interleaved in one process.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/libpbgpu.so
REPS=5 timeout -k 10 300 python3 scripts/ab_lib.py c3_udp_var 33554432 kb24:$L kb20:$L:PBGPU_STAGE_KB=20 kb16_5cu:$L:PBGPU_STAGE_KB=16,PBGPU_WGF=240 kb12_6cu:$L:PBGPU_STAGE_KB=12,PBGPU_WGF=226 > gpurun_out/ab/vst_occ_r02b.txt 2>&1; rc=$?
cat gpurun_out/ab/vst_occ_r02b.txt; exit $rc
