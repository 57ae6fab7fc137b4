#!/bin/bash
# Copy a profile round's evidence (scripts/profile_round.sh output under gpurun_out/prof_$ROUND)
# into profiles/$ROUND/$DEST (default prof/) and profiles/pmc_$ROUND.json.
set -e
cd "$(dirname "$0")/.."
ROUND=${ROUND:-r06}
SRC=gpurun_out/prof_$ROUND
DST=profiles/$ROUND/${DEST:-prof}
rm -rf $DST; mkdir -p $DST/cfg
cp $SRC/bench_under_trace.json $SRC/kernel_trace_summary.json $SRC/pmc_summary.json $SRC/smoke.log $DST/
tail -3 $SRC/pytest.log > $DST/pytest_tail.txt
cp $SRC/bench_trace/run_kernel_stats.csv $DST/rocprofv3_kernel_stats.csv
for f in $SRC/cfg/*.json; do cp $f $DST/cfg/; done
for d in $SRC/cfg/trace_*/; do n=$(basename $d); cp $d/run_kernel_stats.csv $DST/cfg/${n}_kernel_stats.csv; done
python3 scripts/pmc_table.py $SRC $DST/pmc_table.json > /dev/null 2>&1 || true
cp $SRC/pmc_summary.json profiles/pmc_$ROUND.json
ls $DST $DST/cfg
