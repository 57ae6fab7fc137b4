#!/bin/bash
# pb_vstage_kernel L4 sums: group reduction in the payload pass (base) vs per-lane LDS atomics
# folded in the header pass (ldssum); configs[2] at 2^25 frames, then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/variants
REPS=8 timeout -k 10 300 python3 scripts/ab_lib.py c3_udp_var 33554432 base:$L/libpbgpu_new.so ldssum:$L/libpbgpu_ldssum.so > gpurun_out/ab/ldssum_c3.txt 2>&1 || { cat gpurun_out/ab/ldssum_c3.txt; exit 1; }
cat gpurun_out/ab/ldssum_c3.txt
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ab/pytest.log; exit $rc
