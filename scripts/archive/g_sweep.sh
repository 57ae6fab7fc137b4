#!/bin/bash
# lanes-per-frame sweep of the GPF kernel on the large / variable configs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/gsweep; mkdir -p $OUT
for cfg in ${CFGS:-c2_udp_1500 c3_udp_var tcp_all_flags_var}; do
 for g in ${GS:-8 16 32 64}; do
  PBGPU_G=$g timeout -k 10 200 python3 bench.py --steps 8 --warmup 2 --no-variants --cpu-seconds 0 --config $cfg --packets 8388608 > $OUT/${cfg}_$g.json 2>&1 || { echo FAIL $cfg $g; tail -3 $OUT/${cfg}_$g.json; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/${cfg}_$g.json'));print('$cfg G=$g', round(d['value']), 'Mpps', round(d['gbps']), 'GB/s kernel', d['roofline']['achieved'], d['roofline']['kernel'])"
 done
done
