#!/bin/bash
# Round 3: GPU suite; the 64-B host send loop (build -> land in UMEM slots -> TX ring, loopback,
# one TX thread) with the reference's 4,096-slot UMEM and with --umemframes 16384 / 65536.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2k}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
REPS=2 timeout -k 10 500 python -u scripts/e2e_ab.py udp64 1 'u4k:N=33554432' \
    'u16k:N=67108864,ARGS=--umemframes 16384' 'u64k:N=67108864,ARGS=--umemframes 65536' > $O/e2e_udp64_umem.jsonl 2>&1 || exit 1
REPS=1 timeout -k 10 300 python -u scripts/e2e_ab.py udp1500 1 'u4k:' 'u16k:ARGS=--umemframes 16384' \
    > $O/e2e_udp1500_umem.jsonl 2>&1 || exit 1
