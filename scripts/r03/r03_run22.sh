#!/bin/bash
# Round 3: non-temporal stores in pb_xsmall_kernel (64-B UDP, PB_XS_NT=1) vs plain, and the
# library (pb_small_kernel / pb_xpage_kernel non-temporal, PB_SX_NT=1) vs plain on configs[4]'s
# mix and the 98-B / 60-B sequences; span timing, 10 alternating reps; parity of the library.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${OUT:-gpurun_out/r03s2w}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_kat.py -x -q --timeout 120 --timeout-method thread > $O/pytest_nt.log 2>&1 || { tail -20 $O/pytest_nt.log; exit 1; }
tail -2 $O/pytest_nt.log
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
SPAN=1 REPS=10 timeout -k 10 300 python -u scripts/ab_lib.py c2_udp_64 33554432 plain:$L xsnt:$V/libpbgpu_xsnt.so > $O/ab_c2_udp_64_xsnt.jsonl 2>&1 || exit 1
cat $O/ab_c2_udp_64_xsnt.jsonl
for cfg in c4_tcp_syn c5_icmp_echo; do
  SPAN=1 REPS=6 timeout -k 10 300 python -u scripts/ab_lib.py $cfg 33554432 lib:$L sxplain:$V/libpbgpu_sxplain.so > $O/ab_${cfg}_sx.jsonl 2>&1 || exit 1
  echo $cfg; cat $O/ab_${cfg}_sx.jsonl
done
timeout -k 10 200 python3 bench.py --steps 50 --warmup 5 --no-variants --cpu-seconds 0 --config c5_mix > $O/c5_mix.json || exit 1
cat $O/c5_mix.json | cut -c1-400
