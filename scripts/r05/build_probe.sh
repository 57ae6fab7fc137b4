#!/bin/bash
# round-5 A/B probe library (probes/r05_probe.hip: the product's kernels + host shim + probe kernels)
cd "$(dirname "$0")/../.." || exit 1
mkdir -p pb-af-xdp_amd/lib
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -shared \
  -Iinclude -o pb-af-xdp_amd/lib/libpbprobe.so probes/r05_probe.hip "$@"
