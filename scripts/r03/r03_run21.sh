#!/bin/bash
# Round 3: non-temporal stores in pb_small_kernel (98-B ICMP) and pb_xpage_kernel (60-B TCP)
# only (PB_SX_NT=1) vs plain, span timing, 10 alternating reps.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2v}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
for cfg in c4_tcp_syn c5_icmp_echo; do
  SPAN=1 REPS=10 timeout -k 10 300 python -u scripts/ab_lib.py $cfg 33554432 plain:$L sxnt:$V/libpbgpu_sxnt.so > $O/ab_${cfg}_sxnt.jsonl 2>&1 || exit 1
  echo $cfg; cat $O/ab_${cfg}_sxnt.jsonl
done
