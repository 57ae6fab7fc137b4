#!/bin/bash
# Round 3: the 2-mod-4 small frames (98-B ICMP, 106-B UDP).  Alternating A/Bs of the generic
# pb_small_kernel against builds with the frame length as a compile-time constant
# (PB_SMALL_CFLEN, lib/variants) and against the windowed form (PBGPU_SMALL_WIN).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2b}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=6 timeout -k 10 240 python -u scripts/ab_lib.py c5_icmp_echo 33554432 gen:$L c98:$V/libpbgpu_c98.so \
    nomask:$V/libpbgpu_nomask.so w1:$L:PBGPU_SMALL_WIN=1 w4:$L:PBGPU_SMALL_WIN=4 wgt256:$L:PBGPU_SMALL_WGT=256 > $O/ab_icmp98.jsonl 2>&1 || exit 1
REPS=6 timeout -k 10 240 python -u scripts/ab_lib.py c1_udp_static_106 33554432 gen:$L c106:$V/libpbgpu_c106.so nomask:$V/libpbgpu_nomask.so \
    > $O/ab_udp106.jsonl 2>&1 || exit 1
# pb_vline_kernel: full 16-KiB steps without clamps / store guards (PB_VL_SPLIT=1, shipped) vs the
# single guarded loop
REPS=6 timeout -k 10 240 python -u scripts/ab_lib.py c3_udp_var 33554432 split:$L nosplit:$V/libpbgpu_nosplit.so \
    > $O/ab_split_c3.jsonl 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "vline or multi_random or c3_udp_var" -x -q \
    --timeout 120 --timeout-method thread > $O/vline.log 2>&1 || exit 1
