#!/bin/bash
# Round 3: pb_vline_kernel with non-temporal frame stores (PB_VL_NT=1, the library default) vs
# plain stores: parity, alternating A/B, and WRITE_SIZE / FETCH_SIZE of each (one --pmc pass per
# counter and library).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03s2s}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_r03.py -k "vline or c3_udp_var or variable or offsets" -x -q --timeout 120 --timeout-method thread > $O/pytest_vlnt.log 2>&1 || { tail -20 $O/pytest_vlnt.log; exit 1; }
tail -2 $O/pytest_vlnt.log
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=10 timeout -k 10 600 python -u scripts/ab_lib.py c3_udp_var 33554432 nt:$L plain:$V/libpbgpu_vlplain.so > $O/ab_c3_vlnt.jsonl 2>&1 || exit 1
cat $O/ab_c3_vlnt.jsonl
for lib in nt:$L plain:$V/libpbgpu_vlplain.so; do
  for c in WRITE_SIZE FETCH_SIZE; do
    t=${lib%%:*}
    REPS=1 timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${t}_$c -o run -- python3 scripts/ab_lib.py c3_udp_var 33554432 $lib > $O/pmc_${t}_$c.log 2>&1 || { echo "PMC_FAIL $t $c"; tail -5 $O/pmc_${t}_$c.log; exit 1; }
  done
done
echo PMC_DONE
