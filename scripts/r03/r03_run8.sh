#!/bin/bash
# Round 3: GPU suite with per-sequence build streams in span mode, then the configs[4] bench
# line with and without them (PBGPU_SEQ_STREAMS=0), and the default bench line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2h}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --config c5_mix --cpu-seconds 0 --no-variants > $O/c5mix_streams_$r.json 2> $O/c5mix.err || exit 1
  PBGPU_SEQ_STREAMS=0 timeout -k 10 200 python -u bench.py --config c5_mix --cpu-seconds 0 --no-variants > $O/c5mix_serial_$r.json 2> $O/c5mix.err || exit 1
done
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 1
