#!/bin/bash
# PMC passes (one counter group per pass) for one config: CFG, PKTS env
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${CFG:-c2_udp_64}
PKTS=${PKTS:-33554432}
OUT=gpurun_out/pmc_$CFG
mkdir -p $OUT
B="python3 bench.py --steps 5 --warmup 2 --no-variants --cpu-seconds 0 --config $CFG --packets $PKTS"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/trace.log; exit 1; }
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM" "WRITE_SIZE" "FETCH_SIZE"; do
  tag=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$tag -o run -- $B > $OUT/pmc_$tag.log 2>&1 || { echo "PMC_FAIL $grp"; tail -3 $OUT/pmc_$tag.log; }
done
echo done $CFG
