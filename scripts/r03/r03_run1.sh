#!/bin/bash
# Round 3 (session 2) GPU pass: pb_vline_kernel table form parity + A/B, the full GPU suite,
# smoke, the default bench line and per-config lines for configs[2], the 98-B ICMP sequence
# and configs[4].
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "vline or multi_random" -x -q \
    --timeout 120 --timeout-method thread > $O/vline.log 2>&1 || exit 1
REPS=4 timeout -k 10 240 python -u scripts/ab_env.py c3_udp_var 33554432 'lcg:' 'tbl:PBGPU_VL_TBL=1' \
    > $O/ab_tbl_c3.jsonl 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > $O/default.json 2> $O/default.err || exit 1
timeout -k 10 200 python -u bench.py --config c3_udp_var --cpu-seconds 0 --steps 40 > $O/c3.json 2> $O/c3.err || exit 1
timeout -k 10 200 python -u bench.py --config c5_icmp_echo --cpu-seconds 0 > $O/c5icmp.json 2> $O/c5icmp.err || exit 1
timeout -k 10 200 python -u bench.py --config c5_mix --cpu-seconds 0 > $O/c5mix.json 2> $O/c5mix.err || exit 1
