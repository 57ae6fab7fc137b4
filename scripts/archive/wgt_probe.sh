#!/bin/bash
# staged kernel: one-wave workgroups (WGT=64) vs 256-thread ones
set -e
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/wgt_tests.txt 2>&1 || { tail -30 gpurun_out/wgt_tests.txt; exit 1; }
tail -n 1 gpurun_out/wgt_tests.txt
L=${LENS:-1500,1536,1024,512,9000}
LENS=$L timeout -k 10 200 python3 scripts/align_probe.py base > gpurun_out/wgt_base.json
for w in ${WGFS:-16 32 64}; do
  for f in ${FWS:-0 8}; do
    if [ $f = 0 ]; then unset PBGPU_FPW; else export PBGPU_FPW=$f; fi
    PBGPU_WGT=64 PBGPU_WGF=$w LENS=$L timeout -k 10 200 python3 scripts/align_probe.py T64_W${w}_F$f > gpurun_out/wgt_T64_W${w}_F$f.json
  done
done
unset PBGPU_FPW
PBGPU_KERNEL=stage LENS=$L timeout -k 10 200 python3 scripts/align_probe.py var_stage > gpurun_out/wgt_var_stage.json
PBGPU_KERNEL=stage PBGPU_WGT=64 LENS=$L timeout -k 10 200 python3 scripts/align_probe.py var_stage_T64 > gpurun_out/wgt_var_stage_T64.json
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/wgt_*.json")):
    d = json.load(open(f))
    print(d["tag"], "fill", d["fill_gbps"], " ".join(f"{k}={v['gbps']}" for k, v in d.items() if isinstance(v, dict)), d["udp1500"]["kernel"], d["c3_udp_var"]["kernel"])
PY
