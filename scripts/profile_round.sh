#!/bin/bash
# A round's profile evidence on the current tree (ROUND=r05 by default):
#   1. the GPU suite and smoke;
#   2. rocprofv3 --kernel-trace --stats of the default bench command (trace summary of its timed window);
#   3. separate --pmc passes per BASELINE config (WRITE_SIZE / FETCH_SIZE / SQ issue / LDS) ->
#      profiles/pmc_$ROUND.json (HBM bytes per launch: the bench line's roofline.traffic);
#   4. one bench line per config, each under its own --kernel-trace, whose trace summary backs it.
# Output: gpurun_out/prof_$ROUND/ (copied to profiles/$ROUND/prof/ afterwards).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
ROUND=${ROUND:-r06}
OUT=gpurun_out/prof_$ROUND
PMC=profiles/pmc_$ROUND.json
[ -z "$KEEP_OUT" ] && rm -rf $OUT; mkdir -p $OUT/cfg
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  echo "rc=$rc" >> $OUT/pytest.log
  [ $rc -ne 0 ] && { tail -5 $OUT/pytest.log; exit $rc; }
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 1
  echo "tests + smoke ok"
fi
[ -z "$SKIP_TRACE" ] && { timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 100 --warmup 10 --cpu-seconds 2 > $OUT/bench_trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $OUT/bench_trace.log; exit 1; }
grep '^{"metric"' $OUT/bench_trace.log > $OUT/bench_under_trace.json
python3 scripts/trace_summary.py $OUT/bench_trace/run_kernel_trace.csv $OUT/kernel_trace_summary.json
echo "trace done"; }
if [ -z "$SKIP_PMC" ]; then
  for cfg in c2_udp_64 c2_udp_1500 c3_udp_var c4_tcp_syn c5_icmp_echo c5_mix; do
    P=33554432; [ $cfg = c5_mix ] && P=16777216
    B="python3 bench.py --steps 5 --warmup 2 --ramp-seconds 0 --no-variants --cpu-seconds 0 --config $cfg --packets $P"
    for grp in "WRITE_SIZE" "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
      tag=$(echo $grp | cut -d' ' -f1 | tr 'A-Z' 'a-z')
      timeout -s KILL 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_${cfg}_$tag -o run -- $B > $OUT/pmc_${cfg}_$tag.log 2>&1 || { echo "PMC_FAIL $cfg $grp"; tail -3 $OUT/pmc_${cfg}_$tag.log; exit 1; }
    done
    echo "pmc done $cfg"
  done
  python3 scripts/pmc_collect.py $OUT
  cp $OUT/pmc_summary.json $PMC
fi
[ -n "$SKIP_CFG" ] && exit 0
for cfg in c2_udp_64 c2_udp_1500 c3_udp_var c4_tcp_syn c5_icmp_echo c5_mix; do
  V=--no-variants; [ $cfg = c3_udp_var ] && V=
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg/trace_$cfg -o run -- python3 bench.py --steps 50 --warmup 5 $V --cpu-seconds 0 --config $cfg --pmc $PMC > $OUT/cfg/$cfg.log 2>&1 || { echo "CFG_FAIL $cfg"; tail -5 $OUT/cfg/$cfg.log; exit 1; }
  grep '^{"metric"' $OUT/cfg/$cfg.log > $OUT/cfg/$cfg.json
  python3 scripts/trace_summary.py $OUT/cfg/trace_$cfg/run_kernel_trace.csv $OUT/cfg/trace_${cfg}_summary.json 50 > /dev/null
  python3 -c "import json; d=json.load(open('$OUT/cfg/$cfg.json')); r=d['roofline']; t=json.load(open('$OUT/cfg/trace_${cfg}_summary.json'))[0]; print('$cfg', r['kernel'], 'span', r['kernel_ms_avg'], 'trace', round(t['avg_ms'], 5), r['achieved'], 'GB/s', r['frac'], d['write_peak_probe_gbps'], r['traffic'])"
done
