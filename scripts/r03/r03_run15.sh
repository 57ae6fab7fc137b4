#!/bin/bash
# Round 3: pb_vline_kernel with 128-thread workgroups (PBGPU_VL_WGT=128, a build of round 3 that
# was measured and removed: half the region per workgroup, 8-KiB steps) vs 256, and the time
# decomposition (PBGPU_FST_DBG bit 0 prologue alone, bit 1 no stores, bit 2 the stores alone).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2o}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "vline" -x -q --timeout 120 --timeout-method thread > $O/pytest_vline.log 2>&1 || { tail -20 $O/pytest_vline.log; exit 1; }
tail -2 $O/pytest_vline.log
PBGPU_VL_WGT=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_r03.py -k "c3_udp_var or variable or offsets" -x -q --timeout 120 --timeout-method thread > $O/pytest_parity128.log 2>&1 || { tail -20 $O/pytest_parity128.log; exit 1; }
tail -2 $O/pytest_parity128.log
REPS=5 timeout -k 10 400 python -u scripts/ab_env.py c3_udp_var 33554432 w256: w128:PBGPU_VL_WGT=128 \
    w128f100:PBGPU_VL_WGT=128,PBGPU_VL_WGF=100 > $O/ab_c3_wgt.jsonl 2>&1 || exit 1
cat $O/ab_c3_wgt.jsonl
REPS=3 timeout -k 10 400 python -u scripts/ab_env.py c3_udp_var 33554432 full: pro:PBGPU_FST_DBG=1 nost:PBGPU_FST_DBG=2 \
    sto:PBGPU_FST_DBG=4 full128:PBGPU_VL_WGT=128 pro128:PBGPU_VL_WGT=128,PBGPU_FST_DBG=1 \
    nost128:PBGPU_VL_WGT=128,PBGPU_FST_DBG=2 sto128:PBGPU_VL_WGT=128,PBGPU_FST_DBG=4 > $O/ab_c3_decomp.jsonl 2>&1 || exit 1
cat $O/ab_c3_decomp.jsonl
