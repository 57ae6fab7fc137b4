#!/bin/bash
# Round 3: pb_small_kernel's LDS tile sized to its frames (PB_SMALL_DYN=1, a variant build swapped
# in for the library in this scratch copy) vs WGT * NDW dwords (98-B ICMP: 6.2 vs 8.2 KiB per
# workgroup): parity of every kernel shape with the variant, span-timed A/B, configs[4] line.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2z}
mkdir -p $O
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
cp $L /tmp/libpbgpu_static.so && cp $V/libpbgpu_smalldyn.so $L || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dyn.log 2>&1 || { tail -20 $O/pytest_dyn.log; exit 1; }
tail -2 $O/pytest_dyn.log
SPAN=1 REPS=12 timeout -k 10 300 python -u scripts/ab_lib.py c5_icmp_echo 33554432 static:/tmp/libpbgpu_static.so dyn:$L > $O/ab_c5_icmp_echo_dyn.jsonl 2>&1 || exit 1
cat $O/ab_c5_icmp_echo_dyn.jsonl
timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-variants --cpu-seconds 0 --config c5_mix > $O/c5_mix.json || exit 1
python3 -c "import json; d=json.load(open('$O/c5_mix.json')); print('c5_mix', d['ms_per_step'], d['roofline']['frac'])"
# orbit samples every 16th / 8th position (PB_ORB_SH=4 / 3: 4 / 8-MiB tables, walks <= 8 / 4) now
# that the frame stores are non-temporal, against every 32nd (the library)
SPAN=1 REPS=8 timeout -k 10 500 python -u scripts/ab_lib.py c3_udp_var 33554432 sh5:/tmp/libpbgpu_static.so \
    sh4:$V/libpbgpu_sh4.so sh3:$V/libpbgpu_sh3.so > $O/ab_c3_orbsh_nt.jsonl 2>&1 || exit 1
cat $O/ab_c3_orbsh_nt.jsonl
