#!/bin/bash
# Round 3: GPU suite, then pb_xpage_kernel without the 64-bit divisions in its counter tail
# (A/B against the session-start library) and the configs[3] / configs[4] bench lines.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2g}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=8 timeout -k 10 200 python -u scripts/ab_lib.py c4_tcp_syn 33554432 cur:$L base:$V/libpbgpu_base.so \
    > $O/ab_tcp60.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c4_tcp_syn --cpu-seconds 0 > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 200 python -u bench.py --config c5_mix --cpu-seconds 0 > $O/c5mix.json 2> $O/c5mix.err || exit 1
