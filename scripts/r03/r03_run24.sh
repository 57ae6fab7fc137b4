#!/bin/bash
# Round 3: non-temporal stores in pb_fstage_kernel (1500-B UDP, PB_FS_NT=1) vs plain, span timing.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2y}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
SPAN=1 REPS=10 timeout -k 10 400 python -u scripts/ab_lib.py c2_udp_1500 33554432 plain:$L fsnt:$V/libpbgpu_fsnt.so > $O/ab_c2_udp_1500_fsnt.jsonl 2>&1 || exit 1
cat $O/ab_c2_udp_1500_fsnt.jsonl
