#!/bin/bash
# staged-kernel phase timing (diagnostic build with -DPB_TIMING=1)
set -e
mkdir -p gpurun_out
make -s -C pb-af-xdp_amd -B lib/libpbgpu.so HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DPB_TIMING=1"
for kb in ${KBS:-12 24 48}; do
  PBGPU_TIMING=1 PBGPU_STAGE_KB=$kb LENS=1500 timeout -k 10 200 python3 scripts/align_probe.py KB$kb > gpurun_out/tim_KB$kb.json 2> gpurun_out/tim_KB$kb.err
  echo "KB$kb $(cat gpurun_out/tim_KB$kb.json)"
  grep pbgpu_timing gpurun_out/tim_KB$kb.err | sed -n '6p' 
done
