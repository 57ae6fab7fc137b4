#!/bin/bash
# Round 3: the page kernel for 2-mod-4 lengths (PBGPU_XP_FORCE=1: pb_xpage_kernel with the half-
# dword tile writes) — its parity across the small-length sweep, then A/Bs on the 98-B ICMP and
# 106-B UDP frames at 256 / 512 threads; the 64-B page kernel with its length at compile time; the
# 64-B host send loop with larger UMEMs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2j}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
REPS=12 timeout -k 10 240 python -u scripts/ab_lib.py c2_udp_64 33554432 cflen:pb-af-xdp_amd/lib/libpbgpu.so \
    rtlen:pb-af-xdp_amd/lib/variants/libpbgpu_xsrt.so > $O/ab_udp64_cflen.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 240 python -u scripts/ab_env.py c5_icmp_echo 33554432 'lin:' 'xp256:PBGPU_XP_FORCE=1' \
    'xp512:PBGPU_XP_FORCE=1,PBGPU_XP_WGT=512' > $O/ab_icmp98_xpage.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 240 python -u scripts/ab_env.py c1_udp_static_106 33554432 'lin:' 'xp256:PBGPU_XP_FORCE=1' \
    'xp512:PBGPU_XP_FORCE=1,PBGPU_XP_WGT=512' > $O/ab_udp106_xpage.jsonl 2>&1 || exit 1
REPS=2 timeout -k 10 400 python -u scripts/e2e_ab.py udp64 1 'u4k:' 'u16k:ARGS=--umemframes 16384' \
    'u64k:ARGS=--umemframes 65536' > $O/e2e_udp64_umem.jsonl 2>&1 || exit 1
