#!/bin/bash
# Round 3, first GPU pass: pb_vline_kernel / pb_swin_kernel parity, A/Bs against the
# round-2 kernels, the full GPU suite and the default bench line.
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "vline or multi_random or windows" -x -q \
    --timeout 120 --timeout-method thread > $O/vline.log 2>&1 || exit 1
REPS=4 timeout -k 10 240 python -u scripts/ab_env.py c3_udp_var 33554432 'vline:' 'vstage:PBGPU_KERNEL=vstage' \
    > $O/ab_c3.jsonl 2>&1 || exit 1
REPS=4 timeout -k 10 240 python -u scripts/ab_env.py c5_icmp_echo 33554432 'lin:' 'w1:PBGPU_SMALL_WIN=1' \
    'w2:PBGPU_SMALL_WIN=2' 'w4:PBGPU_SMALL_WIN=4' 'w8:PBGPU_SMALL_WIN=8' > $O/ab_icmp.jsonl 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u bench.py --cpu-seconds 6 > $O/default.json 2> $O/default.err
