#!/bin/bash
# Round 3: two bench ranks sharing the GPU over gloo (the N-rank path with real builds), and
# pb_vline_kernel's store shape without its prologue (PBGPU_FST_DBG bit 4) beside the full kernel,
# the prologue alone (bit 0) and the prologue + constant stores (bit 2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2p}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench.py -k "two_ranks or torchrun" -x -v --timeout 170 --timeout-method thread > $O/pytest_ranks.log 2>&1 || { tail -30 $O/pytest_ranks.log; exit 1; }
tail -3 $O/pytest_ranks.log
REPS=4 timeout -k 10 400 python -u scripts/ab_env.py c3_udp_var 33554432 full: pure:PBGPU_FST_DBG=16 sto:PBGPU_FST_DBG=4 \
    pro:PBGPU_FST_DBG=1 > $O/ab_c3_pure.jsonl 2>&1 || exit 1
cat $O/ab_c3_pure.jsonl
