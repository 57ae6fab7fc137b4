#!/bin/bash
# Round 3: GPU suite with XCD-contiguous pb_small_kernel regions, their A/B on the 2-mod-4
# frames, pb_vline_kernel occupancy (PBGPU_LDS_PAD), the configs[4] bench line, and the host
# send loop's landing tunables at 64 B (build -> land in UMEM slots -> TX ring, loopback).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2f}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=10 timeout -k 10 240 python -u scripts/ab_lib.py c5_icmp_echo 33554432 xr:$L lin:$V/libpbgpu_nsmx.so \
    xr_norb:$V/libpbgpu_norb.so > $O/ab_icmp98.jsonl 2>&1 || exit 1
REPS=10 timeout -k 10 240 python -u scripts/ab_lib.py c1_udp_static_106 33554432 xr:$L lin:$V/libpbgpu_nsmx.so \
    > $O/ab_udp106.jsonl 2>&1 || exit 1
REPS=4 timeout -k 10 300 python -u scripts/ab_lib.py c3_udp_var 33554432 occ5:$L occ4:$L:PBGPU_LDS_PAD=5000 \
    occ3:$L:PBGPU_LDS_PAD=14000 > $O/ab_c3_occ.jsonl 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --config c5_mix --cpu-seconds 0 > $O/c5mix.json 2> $O/c5mix.err || exit 1
timeout -k 10 200 python -u bench.py --config c5_icmp_echo --cpu-seconds 0 > $O/c5icmp.json 2> $O/c5icmp.err || exit 1
REPS=2 timeout -k 10 400 python -u scripts/e2e_ab.py udp64 1 'c1024_i3:' 'c2048_i2:PB_LAND_CHUNK=2048,PB_LAND_INFLIGHT=2' \
    'c512_i6:PB_LAND_CHUNK=512,PB_LAND_INFLIGHT=6' 'c256_i12:PB_LAND_CHUNK=256,PB_LAND_INFLIGHT=12' \
    'c1024_nospin:PB_LAND_SPIN=0' > $O/e2e_udp64.jsonl 2>&1 || exit 1
