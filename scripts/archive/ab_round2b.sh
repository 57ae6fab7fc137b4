#!/bin/bash
# Round-2 late A/Bs (profiles/r02/ab): the library before / after the literal-rule change on
# configs[2], the linear small kernel's frames per workgroup on 98-B ICMP and 106-B UDP frames,
# then the whole GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ab
L=pb-af-xdp_amd/lib/variants
REPS=6 timeout -k 10 240 python3 scripts/ab_lib.py c3_udp_var 33554432 old:$L/libpbgpu_old.so new:$L/libpbgpu_new.so > gpurun_out/ab/lit_c3_b.txt 2>&1 || exit 1
cat gpurun_out/ab/lit_c3_b.txt
for cfg in c5_icmp_echo c1_udp_static_106; do
  REPS=6 timeout -k 10 240 python3 scripts/ab_lib.py $cfg 33554432 w64:$L/libpbgpu_new.so w256:$L/libpbgpu_new.so:PBGPU_SMALL_WGT=256 w128:$L/libpbgpu_new.so:PBGPU_SMALL_WGT=128 > gpurun_out/ab/small_wgt_$cfg.txt 2>&1 || exit 1
  cat gpurun_out/ab/small_wgt_$cfg.txt
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/ab/pytest.log; exit $rc
