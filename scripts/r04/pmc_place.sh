#!/bin/bash
# PMC counters per frame buffer (scripts/place_probe.py under rocprofv3 --pmc), one pass per group
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04/pmcplace
mkdir -p $O
CFG=${CFG:-c3_udp_var}; NB=${NB:-4}; K=${K:-5}; KERN=${KERN:-pb_vline_kernel}
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" \
           "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum" \
           "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_sum TCC_TAG_STALL_sum" \
           "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 scripts/place_probe.py $CFG 33554432 $NB $K > $O/p$i.log 2>&1 || { echo "PMC_FAIL $grp"; tail -3 $O/p$i.log; exit 1; }
  grep '"round": 2' $O/p$i.log | cut -c1-100
  python3 scripts/r04/pmc_place.py $O/p$i/run_counter_collection.csv $NB $K 3 $KERN
done
