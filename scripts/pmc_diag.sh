#!/bin/bash
# SQ stall / issue counters of the staged kernels (one rocprofv3 --pmc pass per group)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcdiag; rm -rf $OUT; mkdir -p $OUT
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
G2="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for run in ${DIAG_RUNS:-c3_udp_var:0 c3_udp_var:1 c3_udp_var:2 c2_udp_1500:0}; do
  cfg=${run%%:*}; dbg=${run#*:}
  for g in 1 2; do
    eval grp=\$G$g
    PBGPU_FST_DBG=$dbg timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/${cfg}_d${dbg}_g$g -o run -- python3 bench.py --steps 3 --warmup 1 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $cfg --packets 8388608 > $OUT/${cfg}_d${dbg}_g$g.log 2>&1 || { echo "FAIL $cfg $dbg $g"; tail -5 $OUT/${cfg}_d${dbg}_g$g.log; exit 1; }
  done
  echo done $run
done
python3 - <<'PY'
import csv, glob, collections, os
for d in sorted(glob.glob('gpurun_out/pmcdiag/*_g1')):
    tag = os.path.basename(d)[:-3]
    agg = collections.defaultdict(list)
    for g in (1, 2):
        for f in glob.glob(f'gpurun_out/pmcdiag/{tag}_g{g}/run_counter_collection.csv'):
            for r in csv.DictReader(open(f)):
                if 'stage' in r['Kernel_Name']:
                    agg[r['Counter_Name']].append(float(r['Counter_Value']))
    print(tag, {k: round(sum(v)/len(v)) for k, v in sorted(agg.items())})
PY
