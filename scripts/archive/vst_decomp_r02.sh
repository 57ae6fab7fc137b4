#!/bin/bash
# pb_vstage_kernel time decomposition on configs[2] (2^25 frames; PBGPU_FST_DBG diagnostic
# switches, wrong output): full; store-only (bit 0: no payload / header passes);
# compute-only (bit 1: no stores); structure only (bits 0+1: phase A, windows, order, barriers).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/libpbgpu.so
REPS=5 timeout -k 10 240 python3 scripts/ab_lib.py c3_udp_var 33554432 full:$L store_only:$L:PBGPU_FST_DBG=1 compute_only:$L:PBGPU_FST_DBG=2 structure:$L:PBGPU_FST_DBG=3 > gpurun_out/ab/vst_decomp_r02.txt 2>&1; rc=$?
cat gpurun_out/ab/vst_decomp_r02.txt; exit $rc
