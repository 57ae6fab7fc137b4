#!/bin/bash
# Round 3: pb_orbit_sum's discrete log with its top 12 bits in closed form (PB_ORB_LOG12, the
# library default) vs 24 steps; orbit samples every 16th position (PB_ORB_SH=4: walks <= 8);
# non-temporal frame stores (PB_NT=1, so the stream does not evict the orbit table from L2).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2r}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_r03.py -k "vline or c3_udp_var or variable or offsets" -x -q --timeout 120 --timeout-method thread > $O/pytest_log12.log 2>&1 || { tail -20 $O/pytest_log12.log; exit 1; }
tail -2 $O/pytest_log12.log
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=8 timeout -k 10 600 python -u scripts/ab_lib.py c3_udp_var 33554432 log12:$L log24:$V/libpbgpu_log24.so \
    sh4:$V/libpbgpu_sh4.so nt:$V/libpbgpu_nt.so > $O/ab_c3_log12.jsonl 2>&1 || exit 1
cat $O/ab_c3_log12.jsonl
