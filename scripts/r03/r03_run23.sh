#!/bin/bash
# Round 3: repeat of the non-temporal store A/B for the 98-B ICMP and 64-B UDP kernels with 16
# alternating reps (span timing).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2x}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
SPAN=1 REPS=16 timeout -k 10 300 python -u scripts/ab_lib.py c5_icmp_echo 33554432 lib:$L sxplain:$V/libpbgpu_sxplain.so > $O/ab_c5_icmp_echo_sx16.jsonl 2>&1 || exit 1
cat $O/ab_c5_icmp_echo_sx16.jsonl
SPAN=1 REPS=16 timeout -k 10 300 python -u scripts/ab_lib.py c2_udp_64 33554432 plain:$L xsnt:$V/libpbgpu_xsnt.so > $O/ab_c2_udp_64_xsnt16.jsonl 2>&1 || exit 1
cat $O/ab_c2_udp_64_xsnt16.jsonl
