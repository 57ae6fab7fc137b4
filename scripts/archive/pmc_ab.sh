#!/bin/bash
# PMC A/B of one config under env variants: VARIANTS="tag:VAR=a,VAR2=b ..." CFG PKTS
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
CFG=${CFG:-c2_udp_64}; PKTS=${PKTS:-33554432}
for item in $VARIANTS; do
  tag=${item%%:*}; envs=${item#*:}; [ "$envs" = "$item" ] && envs=""
  OUT=gpurun_out/pmcab_$tag; rm -rf $OUT; mkdir -p $OUT
  B="python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $CFG --packets $PKTS"
  for grp in "${GROUPS1:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT}" "${GROUPS2:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE}"; do
    t=$(echo $grp | cut -d' ' -f1-2 | tr ' ' '_')
    env $(echo $envs | tr ',' ' ') timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$t -o run -- $B > $OUT/pmc_$t.log 2>&1 || { echo "PMC_FAIL $tag $grp"; tail -3 $OUT/pmc_$t.log; exit 1; }
  done
  echo "== $tag"; python3 scripts/pmc_summary.py $OUT pb_ | grep -v "^trace"
done
