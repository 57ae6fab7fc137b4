#!/bin/bash
# staged kernel: frames-per-workgroup sweep (parity at the smallest first)
set -e
mkdir -p gpurun_out
PBGPU_WGF=16 timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/wgf_par16.txt 2>&1 || { tail -40 gpurun_out/wgf_par16.txt; exit 1; }
tail -n 1 gpurun_out/wgf_par16.txt
for w in ${WGFS:-32 64 128 256}; do
  for kb in ${KBS:-24}; do
    PBGPU_WGF=$w PBGPU_STAGE_KB=$kb LENS=${LENS:-1500,1536,1024,512} timeout -k 10 200 python3 scripts/align_probe.py W${w}_KB$kb > gpurun_out/wgf_W${w}_KB$kb.json
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/wgf_W*.json")):
    d = json.load(open(f))
    print(d["tag"], "fill", d["fill_gbps"], " ".join(f"{k}={v['gbps']}" for k, v in d.items() if isinstance(v, dict)), d["udp1500"]["kernel"])
PY
