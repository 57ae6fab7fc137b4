#!/bin/bash
# pb_vline_kernel (configs[2]) and pb_small_kernel (98-B ICMP): time decomposition
# (PBGPU_FST_DBG bit 0: prologue only; bit 1: no stores; diagnostic output) and SQ / TCC
# counters, one rocprofv3 --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03s2c}
mkdir -p $O
REPS=4 timeout -k 10 300 python -u scripts/ab_env.py c3_udp_var 33554432 'full:' \
    'nostore:PBGPU_FST_DBG=2' 'prologue:PBGPU_FST_DBG=1' > $O/decomp_c3.jsonl 2>&1 || exit 1
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
G2="SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR"
G3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"
for cfg in c3_udp_var c5_icmp_echo; do
  B="python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $cfg"
  for g in G1 G2 G3 WRITE_SIZE FETCH_SIZE; do
    eval grp=\${$g:-$g}
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${cfg}_$g -o run -- $B > $O/pmc_${cfg}_$g.log 2>&1 || { echo "PMC_FAIL $cfg $g"; tail -5 $O/pmc_${cfg}_$g.log; exit 1; }
  done
done
echo PMC_DONE
# CIDR table in LDS (PB_RANGE_LDS=1 variant) vs the shipped global / L1 table on configs[3]
# (4 ranges, pb_xpage_kernel): equality, then an alternating A/B
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
timeout -k 10 200 python -u scripts/ab_eq.py $V/libpbgpu_rlds.so > $O/eq_rlds.txt 2>&1 || exit 1
REPS=8 timeout -k 10 240 python -u scripts/ab_lib.py c4_tcp_syn 33554432 l1:$L lds:$V/libpbgpu_rlds.so \
    > $O/ab_cidr_c4.jsonl 2>&1 || exit 1
