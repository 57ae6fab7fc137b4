#!/bin/bash
# Round 3: pb_vline_kernel stores in bursts of 2 / 4 steps (PB_VL_BURST) vs one step at a time.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2n}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=6 timeout -k 10 400 python -u scripts/ab_lib.py c3_udp_var 33554432 b1:$L b2:$V/libpbgpu_burst2.so \
    b4:$V/libpbgpu_burst4.so > $O/ab_c3_burst.jsonl 2>&1 || exit 1
