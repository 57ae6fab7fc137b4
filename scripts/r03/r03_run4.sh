#!/bin/bash
# Round 3: the GPU suite on the new pb_vline_kernel prologue / masks and the small-kernel changes,
# then alternating A/Bs against the session-start library (libpbgpu_base.so) and one switch at a
# time, and a PMC pass of the VALU / SALU / LDS counters.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03s2d}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=5 timeout -k 10 400 python -u scripts/ab_lib.py c3_udp_var 33554432 cur:$L base:$V/libpbgpu_base.so \
    nomt:$V/libpbgpu_nomt.so nobidir:$V/libpbgpu_nobidir.so noimgw:$V/libpbgpu_noimgw.so orb4:$V/libpbgpu_orb4.so \
    orb6:$V/libpbgpu_orb6.so > $O/ab_c3.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 200 python -u scripts/ab_lib.py c5_icmp_echo 33554432 cur:$L base:$V/libpbgpu_base.so \
    > $O/ab_icmp98.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 200 python -u scripts/ab_lib.py c1_udp_static_106 33554432 cur:$L base:$V/libpbgpu_base.so \
    > $O/ab_udp106.jsonl 2>&1 || exit 1
G2="SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR"
G3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES"
for cfg in c3_udp_var c5_icmp_echo; do
  B="python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $cfg"
  for g in G2 G3; do
    eval grp=\${$g:-$g}
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_${cfg}_$g -o run -- $B > $O/pmc_${cfg}_$g.log 2>&1 || { echo "PMC_FAIL $cfg $g"; tail -5 $O/pmc_${cfg}_$g.log; exit 1; }
  done
done
echo PMC_DONE
for v in orb4 orb6; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c3_udp_var_${v}_FETCH_SIZE -o run -- \
      python3 scripts/ab_lib.py c3_udp_var 33554432 $v:$V/libpbgpu_$v.so > $O/pmc_${v}.log 2>&1 || { echo "PMC_FAIL $v"; exit 1; }
done
