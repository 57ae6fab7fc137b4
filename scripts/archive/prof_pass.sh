#!/bin/bash
# rocprofv3: kernel trace + stats, then PMC passes (one counter group per pass)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 2 --no-variants --cpu-seconds 0 ${BENCH_ARGS}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
echo TRACE_OK
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "WRITE_SIZE" "FETCH_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $grp | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$tag -o run -- $B > $OUT/pmc_$tag.log 2>&1 || { echo "PMC_FAIL $grp"; tail -5 $OUT/pmc_$tag.log; }
done
find $OUT -name "*.csv" | head -50
