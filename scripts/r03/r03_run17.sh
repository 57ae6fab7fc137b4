#!/bin/bash
# Round 3: pb_vline_kernel's prologue cost in context: full / without the payload sums' orbit
# reads (PBGPU_FST_DBG bit 5), prologue + constant stores with and without them (bit 2), the
# payload sums in a pass of their own ahead of the build (PBGPU_VL_PSUM=1, a build of round 3 that was
# measured and removed, and its parity), the
# stores alone (bit 4).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2q}
mkdir -p $O
SPAN=1 REPS=6 timeout -k 10 500 python -u scripts/ab_env.py c3_udp_var 33554432 full: noorb:PBGPU_FST_DBG=32 sto:PBGPU_FST_DBG=4 \
    stonoorb:PBGPU_FST_DBG=36 pure:PBGPU_FST_DBG=16 psum:PBGPU_VL_PSUM=1 > $O/ab_c3_orb.jsonl 2>&1 || exit 1
cat $O/ab_c3_orb.jsonl
PBGPU_VL_PSUM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -k "vline or c3_udp_var or variable" -x -q --timeout 120 --timeout-method thread > $O/pytest_psum.log 2>&1 || { tail -20 $O/pytest_psum.log; exit 1; }
tail -2 $O/pytest_psum.log
