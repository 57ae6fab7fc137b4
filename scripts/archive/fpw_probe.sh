#!/bin/bash
# GPF parity at two workgroup sizes, then the lanes-per-frame x frames-per-workgroup sweep
set -e
mkdir -p gpurun_out
timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/fpw_par256.txt 2>&1 || { tail -30 gpurun_out/fpw_par256.txt; exit 1; }
PBGPU_FPW=8 timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/fpw_par8.txt 2>&1 || { tail -30 gpurun_out/fpw_par8.txt; exit 1; }
tail -n 2 gpurun_out/fpw_par256.txt gpurun_out/fpw_par8.txt
for g in ${GS:-8 16 32}; do
  for f in ${FS:-256 64 32 16 8}; do
    PBGPU_G=$g PBGPU_FPW=$f LENS=${LENS:-1500,1536,1024} timeout -k 10 200 python3 scripts/align_probe.py G${g}_F$f > gpurun_out/fpw_G${g}_F$f.json
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/fpw_G*_F*.json")):
    d = json.load(open(f))
    print(d["tag"], "fill", d["fill_gbps"], " ".join(f"{k}={v['gbps']}" for k, v in d.items() if isinstance(v, dict)))
PY
