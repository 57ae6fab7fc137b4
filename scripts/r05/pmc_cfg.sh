#!/bin/bash
# PMC passes (one counter group per run) over one config's short bench (tool only):
#   CFG=c5_icmp_echo TAG=img scripts/r05/pmc_cfg.sh   -> gpurun_out/r05/pmc_$TAG/<group>/
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r05/pmc_$TAG
mkdir -p $OUT
P=33554432; [ "$CFG" = c5_mix ] && P=16777216
B="python3 bench.py --steps 5 --warmup 2 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $CFG --packets $P"
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  tag=$(echo $grp | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/$tag -o run -- $B > $OUT/$tag.log 2>&1 || { echo "PMC_FAIL $grp"; tail -3 $OUT/$tag.log; exit 1; }
done
echo "pmc done $CFG $TAG"
