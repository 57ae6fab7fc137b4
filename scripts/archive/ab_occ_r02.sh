#!/bin/bash
# Workgroups per CU for the small-frame page kernels (dynamic LDS pad, PBGPU_LDS_PAD):
# pb_xsmall_kernel (17 KiB static LDS: 8 per CU unpadded) on configs[1] 64 B, pb_xpage_kernel
# (30 KiB: 5 per CU) on configs[3] 60 B.  Interleaved in one process (scripts/ab_lib.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/libpbgpu.so
REPS=7 timeout -k 10 240 python3 scripts/ab_lib.py c2_udp_64 33554432 p8:$L p7:$L:PBGPU_LDS_PAD=5888 p6:$L:PBGPU_LDS_PAD=9216 p5:$L:PBGPU_LDS_PAD=15360 p4:$L:PBGPU_LDS_PAD=23552 > gpurun_out/ab/occ_xsmall_c2_udp_64.txt 2>&1 || exit 1
cat gpurun_out/ab/occ_xsmall_c2_udp_64.txt
REPS=7 timeout -k 10 240 python3 scripts/ab_lib.py c4_tcp_syn 33554432 p5:$L p4:$L:PBGPU_LDS_PAD=10496 > gpurun_out/ab/occ_xpage_c4_tcp_syn.txt 2>&1 || exit 1
cat gpurun_out/ab/occ_xpage_c4_tcp_syn.txt
