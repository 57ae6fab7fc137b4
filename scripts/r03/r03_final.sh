#!/bin/bash
# Round 3 closing check on the committed tree: the GPU suite, smoke, the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03final}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']
print(d['value'], d['ms_per_step'], r['frac'], r['kernel_ms_avg'], d['udp_1500']['kernel_ms_avg'], d['udp_1500']['roofline_frac'], d['cpu_baseline']['value'], d['cpu_baseline']['cores'])"
