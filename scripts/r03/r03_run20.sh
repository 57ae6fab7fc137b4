#!/bin/bash
# Round 3: non-temporal stores in every kernel (PB_NT=1) vs the library (plain stores except
# pb_vline_kernel's), on the fixed-length configs; span timing (SPAN=1: one event pair per rep).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2u}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
for cfg in c4_tcp_syn c5_icmp_echo c2_udp_64; do
  SPAN=1 REPS=8 timeout -k 10 300 python -u scripts/ab_lib.py $cfg 33554432 lib:$L allnt:$V/libpbgpu_allnt.so > $O/ab_${cfg}_nt_span.jsonl 2>&1 || exit 1
  echo $cfg; cat $O/ab_${cfg}_nt_span.jsonl
done
SPAN=1 REPS=8 timeout -k 10 400 python -u scripts/ab_lib.py c3_udp_var 33554432 lib:$L vlplain:$V/libpbgpu_vlplain.so > $O/ab_c3_udp_var_nt_span.jsonl 2>&1 || exit 1
echo c3_udp_var; cat $O/ab_c3_udp_var_nt_span.jsonl
