#!/bin/bash
# One bench line per BASELINE config (kernel GB/s), plus the write-ceiling sweep of tools/wbench.hip.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/cfg
for cfg in ${CFGS:-c2_udp_64 c2_udp_1500 c3_udp_var c4_tcp_syn c5_icmp_echo}; do
  P=33554432; [ $cfg = c3_udp_var ] && P=16777216
  timeout -k 10 120 python3 bench.py --steps ${STEPS:-50} --warmup 5 --no-variants --cpu-seconds 0 --config $cfg --packets $P > gpurun_out/cfg/$cfg.json || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/cfg/$cfg.json')); r=d['roofline']; print('$cfg', r['kernel'], r['kernel_ms_avg'], r['achieved'], 'GB/s', d['write_peak_probe_gbps'])"
done
if [ -n "$WB" ]; then
  for sz in $WB; do
    timeout -k 10 120 pb-af-xdp_amd/build/wbench $sz sweep > gpurun_out/cfg/wbench_$sz.txt || exit 1
  done
  tail -n 100 gpurun_out/cfg/wbench_*.txt
fi
