#!/bin/bash
# plain vs non-temporal output stores (compile-time PB_NT), frame-length sweep
set -e
mkdir -p gpurun_out
timeout -k 10 240 python3 scripts/align_probe.py nt0 > gpurun_out/align_nt0.json
make -s -C pb-af-xdp_amd -B lib/libpbgpu.so HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -DPB_NT=1"
timeout -k 10 240 python3 scripts/align_probe.py nt1 > gpurun_out/align_nt1.json
cat gpurun_out/align_nt0.json gpurun_out/align_nt1.json
