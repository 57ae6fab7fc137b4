#!/bin/bash
# staged kernel: parity at several (G, F) shapes, then a (G, stage size) sweep
set -e
mkdir -p gpurun_out
run_par() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/stg_par_$tag.txt 2>&1 || { tail -40 gpurun_out/stg_par_$tag.txt; exit 1; }
  tail -n 1 gpurun_out/stg_par_$tag.txt
}
run_par default PBGPU_VERBOSE=0
run_par g8w5 PBGPU_G=8 PBGPU_WGF=5
run_par g64kb4 PBGPU_G=64 PBGPU_STAGE_KB=4
[ -n "$PARITY_ONLY" ] && exit 0
for kb in ${KBS:-12 24 48}; do
  for g in ${GS:-8 16 32}; do
    PBGPU_G=$g PBGPU_STAGE_KB=$kb LENS=${LENS:-1500,1536,1024,512} timeout -k 10 200 python3 scripts/align_probe.py G${g}_KB$kb > gpurun_out/stg_G${g}_KB$kb.json
  done
done
LENS=${LENS:-1500,1536,1024,512} timeout -k 10 200 python3 scripts/align_probe.py default > gpurun_out/stg_default.json
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/stg_*.json")):
    d = json.load(open(f))
    print(d["tag"], "fill", d["fill_gbps"], " ".join(f"{k}={v['gbps']}" for k, v in d.items() if isinstance(v, dict)), d["udp1500"]["kernel"])
PY
