#!/bin/bash
# Round 3: GPU suite with 4-B packed offsets (pb_vline_kernel) and their A/B against the
# 8-B offsets of the previous build, with a WRITE_SIZE pass of each.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${OUT:-gpurun_out/r03s2i}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
echo "rc=$rc" >> $O/pytest.log
[ $rc -ne 0 ] && exit $rc
L=pb-af-xdp_amd/lib/libpbgpu.so
V=pb-af-xdp_amd/lib/variants
REPS=6 timeout -k 10 300 python -u scripts/ab_lib.py c3_udp_var 33554432 off32:$L off64:$V/libpbgpu_u64.so \
    > $O/ab_c3_off32.jsonl 2>&1 || exit 1
for v in off32:$L off64:$V/libpbgpu_u64.so; do
  t=${v%%:*}
  REPS=1 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c3_udp_var_${t}_WRITE_SIZE -o run -- \
      python3 scripts/ab_lib.py c3_udp_var 33554432 $v > $O/pmc_$t.log 2>&1 || { echo "PMC_FAIL $t"; exit 1; }
done
