#!/bin/bash
# pb_vline_kernel: time decomposition (PBGPU_FST_DBG bit 0 no payload generation, bit 1 no
# stores; diagnostic output) and SQ / TCC counters, one rocprofv3 --pmc pass per group
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03d}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "vline or multi_random or c3_udp_var or counters" -x -q \
    --timeout 120 --timeout-method thread > $O/vline.log 2>&1 || exit 1
REPS=3 timeout -k 10 300 python -u scripts/ab_env.py c3_udp_var 33554432 'full:' \
    'nostore:PBGPU_FST_DBG=2' 'vstage:PBGPU_KERNEL=vstage' 'w192:PBGPU_VL_WGF=192' > $O/decomp.jsonl 2>&1 || exit 1
B="python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config c3_udp_var"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
G2="SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR"
G3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for g in G1 G2 G3 WRITE_SIZE FETCH_SIZE; do
  eval grp=\${$g:-$g}
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/pmc_$g -o run -- $B > $O/pmc_$g.log 2>&1 || { echo "PMC_FAIL $g"; tail -5 $O/pmc_$g.log; exit 1; }
done
echo PMC_DONE
