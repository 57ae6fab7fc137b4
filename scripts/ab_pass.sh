#!/bin/bash
# A/B of kernel options in one box session + PMC summary of the 64-B small kernel
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/ab
mkdir -p $OUT
B="python3 bench.py --steps 20 --warmup 3 --no-variants --cpu-seconds 0"
for nt in 0 1 0 1; do
  PBGPU_NT=$nt timeout -k 10 120 $B > $OUT/nt$nt.json 2>&1 || { echo FAIL; cat $OUT/nt$nt.json; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/nt$nt.json'));print('NT=$nt', d['value'], d['roofline']['achieved'], d['roofline']['kernel_ms_avg'])"
done
for cfg in c4_tcp_syn c2_udp_1500 c3_udp_var c5_icmp_echo; do
  timeout -k 10 200 $B --config $cfg --packets 8388608 > $OUT/$cfg.json 2>&1 || { echo FAIL $cfg; tail -5 $OUT/$cfg.json; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$cfg.json'));print('$cfg', d['value'], 'Mpps', d['gbps'], 'GB/s kernel', d['roofline']['achieved'])"
done
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$tag -o run -- $B --steps 5 > $OUT/pmc_$tag.log 2>&1 || { echo "PMC_FAIL $grp"; tail -3 $OUT/pmc_$tag.log; }
done
echo done
