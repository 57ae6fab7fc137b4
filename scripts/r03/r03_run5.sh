#!/bin/bash
# Round 3: GPU suite, then A/Bs: pb_vline_kernel region size (PBGPU_VL_WGF) and per-step
# workgroup sync (PB_VL_SYNC); pb_small_kernel batched tile reads (PB_SMALL_RBATCH) and XCD-
# contiguous regions (PB_SMALL_XREMAP); pb_xsmall_kernel XCD-contiguous pages (PB_XS_XREMAP).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2e}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=5 timeout -k 10 400 python -u scripts/ab_lib.py c3_udp_var 33554432 cur:$L sync:$V/libpbgpu_sync.so \
    w128:$L:PBGPU_VL_WGF=128 w96:$L:PBGPU_VL_WGF=96 w64:$L:PBGPU_VL_WGF=64 > $O/ab_c3.jsonl 2>&1 || exit 1
REPS=8 timeout -k 10 200 python -u scripts/ab_lib.py c5_icmp_echo 33554432 cur:$L norb:$V/libpbgpu_norb.so \
    smx:$V/libpbgpu_smx.so base:$V/libpbgpu_base.so > $O/ab_icmp98.jsonl 2>&1 || exit 1
REPS=12 timeout -k 10 200 python -u scripts/ab_lib.py c2_udp_64 33554432 cur:$L xsx:$V/libpbgpu_xsx.so \
    > $O/ab_udp64_xsx.jsonl 2>&1 || exit 1
